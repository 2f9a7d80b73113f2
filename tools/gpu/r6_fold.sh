#!/bin/bash
# Round 6: the k-means++ fold (first Lloyd E-step in the last k-means++ pass):
# same bits (fit fingerprint with and without it, against the recorded one),
# the fit tests, kernel stats, and the bench with / without (alternating).
set -o pipefail
TAG=${1:-r6fold}
EXP=${2:-}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for v in 1 0; do
  MW_KPP_FOLD=$v timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_$v.txt" 2>&1 || { tail -5 "$OUT/fp_$v.txt"; exit 1; }
  echo "FOLD=$v $(grep FP "$OUT/fp_$v.txt")"
  if [ -n "$EXP" ]; then grep -q "$EXP" "$OUT/fp_$v.txt" && echo "  same as recorded" || echo "  DIFFERS from recorded"; fi
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "kmeans or c_fit or end_to_end or hard256 or smoke or config2 or kinds or st_labeler" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" ) || { tail -5 "$OUT/bench_prof.err"; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "kpp" in n or "lloyd" in n:
        print(f"{n[:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
for v in 1 0 1 0; do
  MW_KPP_FOLD=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-outputs > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { tail -5 "$OUT/bench_$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('FOLD=$v', round(d['ms_per_step'],3), 'fit', d['kernels']['kmeans_fit']['mean_ms'], 'design', round(d['design_point']['ms_per_step'],3), d['design_point']['kmeans_fit_ms'])"
done
echo "[r6_fold] done"
