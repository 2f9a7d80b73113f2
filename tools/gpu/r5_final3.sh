#!/bin/bash
# Round-5 final tree after the Lloyd grid change: smoke(), the default bench
# (headline + design point + CPU baseline), rocprofv3 kernel statistics at
# config 2 (the GPU suite ran on this tree in r5_gridval.sh)
set -o pipefail
TAG=${1:-r5final3}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" ) || exit 1
echo "[final3] done"
