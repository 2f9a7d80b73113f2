#!/bin/bash
# config-5 share fit history per list-pass variant library (tools/probe/liblist_<V>.so)
#   VARIANTS="PAD" bash tools/gpu/r5_listvar.sh out
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-listvar}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
summ='import json,sys; d=json.load(open(sys.argv[1])); L=[t[2] for t in d["launches"] if t[0]=="list"]; print(sys.argv[2], "wall", round(d["wall_s"],3), "n_iter", d["n_iter"], "list", len(L), round(sum(L),1))'
for v in main $VARIANTS; do
  L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
  timeout -k 10 500 env ${L:+MW_LIB=$L} python -u tools/gpu/r5_c5fitdiag.py > "$OUT/diag_$v.json" 2> "$OUT/diag_$v.err" || { tail -5 "$OUT/diag_$v.err"; exit 1; }
  python -c "$summ" "$OUT/diag_$v.json" $v
done
echo "[listvar] done"
