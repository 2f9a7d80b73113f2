#!/bin/bash
# Round-4 A/B: k-means++ tile sums by a lane-0 wave sum with DPP row shifts
# (new lib) against the committed lib (abv/lib_head.so): k-means++ index
# tests (goldens, wide rows, full size), config 2 x2 and config 5 x1 alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4dpp}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lloyd_kinds.py tests/test_gpu_fit_c.py -x -q --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_new$r.json 2> $OUT/c2_new$r.err || exit 1
  MW_LIB=abv/lib_head.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_head$r.json 2> $OUT/c2_head$r.err || exit 1
done
timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_new.json 2> $OUT/c5_new.err || exit 1
MW_LIB=abv/lib_head.so timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_head.json 2> $OUT/c5_head.err || exit 1
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$R/$OUT/prof_c2.json" 2> "$R/$OUT/prof_c2.err" ) || exit 1
echo "[dpp] done"
