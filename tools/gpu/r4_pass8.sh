#!/bin/bash
# Round-4 GPU pass 8: k-means++ pass at F > 32 with per-tile table pointers
# (no hoisted table, fewer SGPR spills): k-means++ index parity, config 5 / 2.
set -o pipefail
TAG=${1:-r4i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -v --timeout 300 $T -m gpu -k "kpp or kmeans or plusplus" > $OUT/kpp.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2.json 2> $OUT/c2.err || exit 1
echo "[pass8] done"; exit 0
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err" ) || exit 1
echo "[pass8] done"
