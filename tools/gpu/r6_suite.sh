#!/bin/bash
# Round 6: the GPU suite (changed tests first, then everything), smoke(), the
# default bench.  Each step under its own limit; stop at the first failure.
set -o pipefail
TAG=${1:-r6a}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
FIRST=${FIRST:-"tests/test_gpu_stream.py tests/test_gpu_dist.py tests/test_gpu_nccl.py tests/test_gpu_parity.py tests/test_gpu_lloyd_kinds.py"}
timeout -k 10 900 python -u -m pytest $FIRST -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_first.log" 2>&1 || { tail -40 "$OUT/pytest_first.log"; exit 1; }
tail -3 "$OUT/pytest_first.log"
if [ -z "$NOFULL" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'])"
echo "[r6_suite] done"
