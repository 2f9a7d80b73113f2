#!/bin/bash
# host-side profile of the config-2 timed steps (cProfile of bench.py's timed loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4m}; mkdir -p $OUT
MW_BENCH_CPROFILE=$OUT/cprof timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2.json 2> $OUT/c2.err || exit 1
echo "[hostprof] done"
