#!/bin/bash
# config-5 share A/B: MW_DRAWS_BESIDE=0 vs 1
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-c5ab}"; mkdir -p "$OUT"; cd "$R" || exit 1
for v in 0 1; do
  MW_DRAWS_BESIDE=$v timeout -k 10 500 python -u bench.py --slides-per-gpu 4 --size 40000 --channels 50 --source synth --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/b_$v.json" 2> "$OUT/b_$v.err" || { tail -5 "$OUT/b_$v.err"; exit 1; }
done
echo done
