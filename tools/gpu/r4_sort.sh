#!/bin/bash
# sweep in slide row order: exactness (sweep tests) and A/B against draw order
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4o}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu -k "sweep or optimal or batched or pass_kinds" > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  MW_SWEEP_SORT=0 timeout -k 10 300 python -u bench.py --sweep --steps 3 --warmup 1 --no-cpu-baseline > $OUT/sw_draw_$r.json 2> $OUT/sw_draw_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --sweep --steps 3 --warmup 1 --no-cpu-baseline > $OUT/sw_sort_$r.json 2> $OUT/sw_sort_$r.err || exit 1
done
echo "[sort] done"
