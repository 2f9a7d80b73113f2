#!/bin/bash
# Round 6: k-means++ pass with two tiles in flight per wave (MW_KPP_PF=2: 4
# waves per SIMD with spills, 3: 3 waves per SIMD) vs one (1): same bits
# (fit fingerprint) and kernel time (rocprofv3 stats over the bench).
set -o pipefail
TAG=${1:-r6kpppf}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for pf in 1 2 3; do
  MW_KPP_PF=$pf timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_$pf.txt" 2>&1 || { tail -5 "$OUT/fp_$pf.txt"; exit 1; }
  grep FP "$OUT/fp_$pf.txt"
done
for pf in 1 2 3 1; do
  ( cd /tmp && export TMPDIR=/tmp && MW_KPP_PF=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$pf" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_$pf.json" 2> "$OUT/bench_$pf.err" ) || { tail -5 "$OUT/bench_$pf.err"; exit 1; }
  ST=$(find "$OUT/prof_$pf" -name "*kernel_stats.csv" | head -1)
  echo "PF=$pf $(python -c "import json; d=json.load(open('$OUT/bench_$pf.json')); print(round(d['ms_per_step'],3), d['kernels']['kmeans_fit']['mean_ms'])")"
  grep "kpp_pass" "$ST" | cut -d, -f1-4 | sed 's/(float const.*"//'
done
echo "[r6_kpppf] done"
