#!/bin/bash
# Round-4 A/B: the config-2 first Lloyd pass at three waves per SIMD (MW_LLOYD_FIRST_W3=1)
# against the unbounded instance (default), same library: the
# bitwise test, config 2 x2 alternating, the design point.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4w3}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -q --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  MW_LLOYD_FIRST_W3=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_w3_$r.json 2> $OUT/c2_w3_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_w2_$r.json 2> $OUT/c2_w2_$r.err || exit 1
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && MW_LLOYD_FIRST_W3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$R/$OUT/prof_c2.json" 2> "$R/$OUT/prof_c2.err" ) || exit 1
echo "[w3] done"
