#!/bin/bash
# Round-4 GPU pass 6: fp32 fixed-point conversion in the Lloyd M-steps --
# kinds + parity + full-size exactness, config 2 / 5 timing.
set -o pipefail
TAG=${1:-r4g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline"
B5="--size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -v --timeout 300 $T -m gpu > $OUT/kinds_parity.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $B > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 300 python -u bench.py $B5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 800 $T -m gpu > $OUT/fullsize.log 2>&1 || exit 1
echo "[pass6] done"
