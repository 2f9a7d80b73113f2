#!/bin/bash
# config-2 A/B of two env settings ($AB_A / $AB_B), alternating, then the full GPU suite
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-ab2}"; mkdir -p "$OUT"; cd "$R" || exit 1
for i in 1 2; do
  for v in A B; do
    E=$([ $v = A ] && echo "$AB_A" || echo "$AB_B")
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --no-design-point > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err" || { tail -5 "$OUT/b_${v}_$i.err"; exit 1; }
  done
done
if [ -n "$FULL" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
fi
echo "[ab2] done"
