#!/bin/bash
# Round 6: blur band height A/B (tile-count quantisation of the band grid):
# blur-only timing per band height, then the default bench at three heights.
set -o pipefail
TAG=${1:-r6bh}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/blur_bench.py 10000 30 "MW_BLUR_BH=512,MW_BLUR_BH=770,MW_BLUR_BH=625,MW_BLUR_BH=527,MW_BLUR_BH=400,MW_BLUR_BH=1000,MW_BLUR_BH=512,MW_BLUR_BH=770" > "$OUT/blur_bh.txt" 2>&1 || { tail -5 "$OUT/blur_bh.txt"; exit 1; }
cat "$OUT/blur_bh.txt"
for bh in 512 770 625 512 770 625; do
  MW_BLUR_BH=$bh timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_bh$bh.json" 2> "$OUT/bench_bh$bh.err" || { tail -5 "$OUT/bench_bh$bh.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_bh$bh.json')); print('BH=$bh', round(d['ms_per_step'],3), d['kernels']['blur']['mean_ms'], d['kernels']['kmeans_fit']['mean_ms'])"
done
echo "[r6_blurbh] done"
