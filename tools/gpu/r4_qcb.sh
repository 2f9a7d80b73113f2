#!/bin/bash
# Round-4: label-pass QC against the estimators' passes, config 2 and config 5 slides
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qcb}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/qc_label_bench.py --size 10000 --channels 30 > $OUT/qc_c2.json 2> $OUT/qc_c2.err || exit 1
timeout -k 10 700 python -u tools/qc_label_bench.py --size 40000 --channels 50 --reps 2 > $OUT/qc_c5.json 2> $OUT/qc_c5.err || exit 1
echo "[qcb] done"
