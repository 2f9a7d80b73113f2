#!/bin/bash
# Round 6: interleaved tile mapping A/B (MW_ASSIGN_IL) in the bench step, with
# the label/confidence maps and domain records compared bitwise
set -o pipefail
TAG=${1:-r6il}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for v in 0 1; do
  MW_ASSIGN_IL=$v timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_$v.txt" 2>&1 || { tail -5 "$OUT/fp_$v.txt"; exit 1; }
  echo "IL=$v $(grep FP "$OUT/fp_$v.txt")"
done
MW_ASSIGN_IL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "assign or label or conf or domain or qc or end_to_end or hard256" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in 0 1 0 1; do
  MW_ASSIGN_IL=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { tail -5 "$OUT/bench_$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('IL=$v', round(d['ms_per_step'],3), {k: v['mean_ms'] for k, v in d['kernels'].items()})"
done
echo "[r6_il] done"
