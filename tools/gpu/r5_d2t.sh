#!/bin/bash
# dense2 exactness tests + default-config sweep
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-d2t}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
timeout -k 10 200 python -u bench.py --sweep --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/sw.json" 2> "$OUT/sw.err" || { tail -5 "$OUT/sw.err"; exit 1; }
echo "[d2t] done"
