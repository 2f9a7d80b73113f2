#!/bin/bash
# Round-4 final tree (after the FMAX = 52 instances): the whole GPU suite,
# smoke(), the default bench, the config-5 slice and the two-slide cohort line.
set -o pipefail
TAG=${1:-r4final5}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || { tail -5 "$OUT/c5.err"; exit 1; }
timeout -k 10 400 python -u bench.py --size 40000 --channels 50 --slides-per-gpu 2 --source synth --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5x2.json" 2> "$OUT/c5x2.err" || { tail -5 "$OUT/c5x2.err"; exit 1; }
echo "[final5] done"
