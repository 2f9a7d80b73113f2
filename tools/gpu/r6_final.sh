#!/bin/bash
# Round 6 evidence for the tree as it stands: the whole GPU suite, smoke(),
# the default bench line, rocprofv3 kernel stats of the bench, the PMC
# passes (SQ, MFMA, FETCH, WRITE) for the roofline's traffic and counters.
set -o pipefail
TAG=${1:-r6final}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" ) || { tail -5 "$OUT/bench_prof.err"; exit 1; }
TAG=${TAG}_c2 BENCH_ARGS="--no-design-point" PMC_PASSES=sq,mfma,fetch,write bash "$R/tools/gpu/pmc_bench.sh" > "$OUT/pmc_c2.log" 2>&1 || { tail -5 "$OUT/pmc_c2.log"; exit 1; }
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_source'))"
echo "[r6_final] done"
