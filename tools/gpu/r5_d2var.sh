#!/bin/bash
# dense2 timing variants (tools/probe/d2_variants.sh) through the per-launch probe
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-d2var}"; mkdir -p "$OUT"; cd "$R" || exit 1
for ks in "9,10,11,12,13,14,15,16,17,18,19,20" "18,19,20"; do
  for v in default ${VARIANTS:-noclose noflush bonly lonly}; do
    lib="$R/tools/probe/libd2_$v.so"; [ "$v" = default ] && lib="$R/milwrm_amd/libmilwrm_amd.so"
    D2_KS=$ks MW_LIB="$lib" timeout -k 10 120 python -u tools/probe/d2_bench.py >> "$OUT/var.jsonl" 2>> "$OUT/var.err" || { tail -5 "$OUT/var.err"; exit 1; }
  done
done
echo done
