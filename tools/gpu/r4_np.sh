#!/bin/bash
# Round-4 A/B: distance loops bounded to the row's own feature pairs at
# FMAX = 64 (new lib) against the committed lib (abv/lib_head.so):
# kinds + parity tests for exactness, then config 5 / config 2 benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4np}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -q --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_new$r.json 2> $OUT/c5_new$r.err || exit 1
  MW_LIB=abv/lib_head.so timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_head$r.json 2> $OUT/c5_head$r.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_new$r.json 2> $OUT/c2_new$r.err || exit 1
  MW_LIB=abv/lib_head.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_head$r.json 2> $OUT/c2_head$r.err || exit 1
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err" ) || exit 1
echo "[np] done"
