#!/bin/bash
# Round 6: 128-column blur bands (MW_BLUR_BT8=1) vs 64: blur alone (bitwise
# cross-check) and inside the bench step, alternating.
set -o pipefail
TAG=${1:-r6bt8}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for v in 0 1 0 1; do
  BLUR_SAVE="$OUT/blur_$v.npy" MW_BLUR_BT8=$v timeout -k 10 300 python -u tools/blur_bench.py 10000 30 "MW_BLUR_BH=512" > "$OUT/blur_$v.txt" 2>&1 || { tail -5 "$OUT/blur_$v.txt"; exit 1; }
  echo "BT8=$v $(grep 'BW=' "$OUT/blur_$v.txt")"
done
python -c "import numpy as np; a=np.load('$OUT/blur_0.npy'); b=np.load('$OUT/blur_1.npy'); print('bitwise equal samples:', np.array_equal(a, b))"
for v in 0 1 0 1; do
  MW_BLUR_BT8=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { tail -5 "$OUT/bench_$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('BT8=$v', round(d['ms_per_step'],3), {k: v['mean_ms'] for k, v in d['kernels'].items()})"
done
echo "[r6_bt8] done"
