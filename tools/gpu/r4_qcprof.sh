#!/bin/bash
# Round-4: kernel stats of the label-pass QC bench (config 2 and config 5 slides)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qcp}; mkdir -p $OUT
R="$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/c2" -o c2 -- python "$R/tools/qc_label_bench.py" --size 10000 --channels 30 --reps 1 > "$R/$OUT/c2.json" 2> "$R/$OUT/c2.err" ) || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/c5" -o c5 -- python "$R/tools/qc_label_bench.py" --size 40000 --channels 50 --reps 1 > "$R/$OUT/c5.json" 2> "$R/$OUT/c5.err" ) || exit 1
echo "[qcprof] done"
