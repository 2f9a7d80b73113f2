#!/bin/bash
# Round-5 final tree, part B: PMC passes (config 2: SQ, MFMA, FETCH, WRITE;
# the config-5 slice: FETCH, WRITE) for tools/pmc_traffic.py, the config-5
# slice under rocprofv3 stats, and the config-5 4-slide share line.
set -o pipefail
TAG=${1:-r5finalB}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
TAG=${TAG}_c2 BENCH_ARGS="--no-design-point" PMC_PASSES=sq,sq2,mfma,fetch,write bash "$R/tools/gpu/pmc_bench.sh" > "$OUT/pmc_c2.log" 2>&1 || { tail -5 "$OUT/pmc_c2.log"; exit 1; }
TAG=${TAG}_c5 BENCH_ARGS="--size 40000 --channels 50" PMC_PASSES=fetch,write bash "$R/tools/gpu/pmc_bench.sh" > "$OUT/pmc_c5.log" 2>&1 || { tail -5 "$OUT/pmc_c5.log"; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err" ) || exit 1
echo "[finalB] done"
