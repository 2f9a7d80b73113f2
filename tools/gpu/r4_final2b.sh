#!/bin/bash
# Round-4 final tree, part 2: rocprofv3 kernel statistics (config 2, config 5)
# and the PMC passes (config 2: SQ, SQ2, MFMA, FETCH, WRITE; config 5: FETCH,
# WRITE) behind bench.py's roofline.traffic.
set -o pipefail
TAG=${1:-r4final2}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" ) || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err" ) || exit 1
TAG=${TAG}_c2 BENCH_ARGS="--no-design-point" PMC_PASSES=sq,sq2,mfma,fetch,write bash "$R/tools/gpu/pmc_bench.sh" || exit 1
TAG=${TAG}_c5 BENCH_ARGS="--size 40000 --channels 50" PMC_PASSES=fetch,write bash "$R/tools/gpu/pmc_bench.sh" || exit 1
echo "[final2b] done"
