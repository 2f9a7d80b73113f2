#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-d2var}"; mkdir -p "$OUT"; cd "$R" || exit 1
for v in base noclose nokeys noflush; do
  MW_LIB="$R/tools/probe/libd2_$v.so" timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/var.jsonl" 2>> "$OUT/var.err" || { tail -5 "$OUT/var.err"; exit 1; }
done
D2_KS=9,11,13,15,17,19 MW_LIB="$R/tools/probe/libd2_base.so" timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/var.jsonl" 2>> "$OUT/var.err" || exit 1
D2_KS=18,19,20 MW_LIB="$R/tools/probe/libd2_base.so" timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/var.jsonl" 2>> "$OUT/var.err" || exit 1
echo done
