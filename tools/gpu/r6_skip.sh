#!/bin/bash
# k-means++ passes with skipped cur stores: fit fingerprint with and without
# (MW_KPP_SKIP_STORE=0), the k-means++ / fit GPU tests, then same-box kernel
# stats and step times, alternating.
set -o pipefail
TAG=${1:-r6skip}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for v in 1 0; do
  MW_KPP_SKIP_STORE=$v timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_$v.txt" 2>&1 || { tail -5 "$OUT/fp_$v.txt"; exit 1; }
  echo "skip=$v $(grep -o 'n_iter=[0-9]* inertia=[0-9.]*' "$OUT/fp_$v.txt") $(grep -o 'sha1=.*' "$OUT/fp_$v.txt")"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "kpp or kmeans or fit or parity or lloyd or fullsize or dist or nccl or sweep" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in 1 0; do
  ( cd /tmp && export TMPDIR=/tmp MW_KPP_SKIP_STORE=$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof_$v.json" 2> "$OUT/bench_prof_$v.err" ) || { tail -5 "$OUT/bench_prof_$v.err"; exit 1; }
done
for rep in 1 2; do
  for v in 1 0; do
    MW_KPP_SKIP_STORE=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || { tail -5 "$OUT/bench_${v}_$rep.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$rep.json')); print('skip=$v', $rep, round(d['ms_per_step'], 3), d['kernels']['kmeans_fit']['mean_ms'])"
  done
done
python - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
for v in ("1", "0"):
    f = glob.glob(f"{out}/prof_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "kpp_" in r["Name"]:
            print(v, f"{r['Name'][:48]:48s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:8.1f} us")
PY
echo "[r6_skip] done"
