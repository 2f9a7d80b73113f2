#!/bin/bash
# Round-5 final tree, part A: the whole GPU suite, smoke(), the default bench
# (headline + design point + CPU baseline), the sweep bench, rocprofv3 kernel
# statistics at config 2 and the config-5 slice.  Stops at the first failure.
set -o pipefail
TAG=${1:-r5finalA}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider --durations=15 > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
timeout -k 10 200 python -u bench.py --sweep --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/sweep.json" 2> "$OUT/sweep.err" || { tail -5 "$OUT/sweep.err"; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" ) || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_sw" -o sw -- python "$R/bench.py" --sweep --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_sw.json" 2> "$OUT/prof_sw.err" ) || exit 1
echo "[finalA] done"
