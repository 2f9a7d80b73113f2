#!/bin/bash
# Round-4 final-tree pass: the whole GPU suite, smoke(), the default bench
# (headline + design point + CPU baseline), the sweep bench, rocprofv3 kernel
# statistics, PMC passes (config 2: SQ, MFMA, FETCH, WRITE; config 5: FETCH,
# WRITE).  Each step under its own limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r4final}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 python -u bench.py --sweep --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/sweep.json" 2> "$OUT/sweep.err" || { tail -5 "$OUT/sweep.err"; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" ) || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err" ) || exit 1
TAG=${TAG}_c2 BENCH_ARGS="--no-design-point" PMC_PASSES=sq,sq2,mfma,fetch,write bash "$R/tools/gpu/pmc_bench.sh" || exit 1
TAG=${TAG}_c5 BENCH_ARGS="--size 40000 --channels 50" PMC_PASSES=fetch,write bash "$R/tools/gpu/pmc_bench.sh" || exit 1
echo "[final] done"
