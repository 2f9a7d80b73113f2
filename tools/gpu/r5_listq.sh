#!/bin/bash
# list-pass recompute queue: exactness tests, config-5 share fit timing, config-2 bench
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-listq}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
timeout -k 10 900 python -u tools/gpu/r5_c5fitdiag.py > "$OUT/diag.json" 2> "$OUT/diag.err" || { tail -5 "$OUT/diag.err"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
echo "[listq] done"
