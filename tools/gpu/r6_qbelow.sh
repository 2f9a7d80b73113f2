#!/bin/bash
# Same-box sweep of the Lloyd pass-kind threshold (MW_LLOYD_QUEUE_BELOW: a pass
# takes the full-tile kind while the previous pass recomputed more than this
# fraction of the rows, else the marked-list kind): fit fingerprint and step
# time per value, two rounds.
set -o pipefail
TAG=${1:-r6qb}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
QS=${QS:-0.3 0.5 0.7 0.9}
for q in $QS; do
  MW_LLOYD_QUEUE_BELOW=$q timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_$q.txt" 2>&1 || { tail -5 "$OUT/fp_$q.txt"; exit 1; }
  echo "q=$q $(grep FP "$OUT/fp_$q.txt" | cut -c1-60) $(grep -o 'sha1=.*' "$OUT/fp_$q.txt")"
done
for rep in 1 2; do
  for q in $QS; do
    MW_LLOYD_QUEUE_BELOW=$q timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_${q}_$rep.json" 2> "$OUT/bench_${q}_$rep.err" || { tail -5 "$OUT/bench_${q}_$rep.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${q}_$rep.json')); print('q=$q', $rep, round(d['ms_per_step'], 3), d['kernels']['kmeans_fit']['mean_ms'])"
  done
done
echo "[r6_qbelow] done"
