#!/bin/bash
# Round-4 A/B: k-means++ at even F > 32 with the candidate table in LDS (new
# lib) against the committed lib (abv/lib_head.so): k-means++ index tests,
# config 5 x2 alternating, kernel statistics.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4kppl}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 700 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_fullsize.py -x -v --timeout 600 $T -m gpu -k "kpp or fm52 or config5" > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_new$r.json 2> $OUT/c5_new$r.err || exit 1
  MW_LIB=abv/lib_head.so timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_head$r.json 2> $OUT/c5_head$r.err || exit 1
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err" ) || exit 1
echo "[kppl] done"
