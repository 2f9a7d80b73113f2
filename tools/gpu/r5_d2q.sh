#!/bin/bash
# dense2 quick round: exactness tests, per-launch probe, default sweep
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-d2q}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/probe.jsonl" 2>> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
D2_KS=18,19,20 timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/probe.jsonl" 2>> "$OUT/probe.err" || exit 1
timeout -k 10 200 python -u bench.py --sweep --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/sw.json" 2> "$OUT/sw.err" || { tail -5 "$OUT/sw.err"; exit 1; }
echo "[d2q] done"
