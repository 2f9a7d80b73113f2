#!/bin/bash
# list-pass gather depth A/B (lib_G16 / lib_G32 against the main library):
# (the variant libraries were built with -DMW_LIST_GB=16/32, a gather-depth macro since reverted)
# pass-kind exactness on G32, then the config-5 share fit history per library
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-listgb}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
MW_LIB="$R/tools/probe/liblist_G32.so" timeout -k 10 400 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
tail -1 "$OUT/kinds.log"
summ='import json,sys; d=json.load(open(sys.argv[1])); L=[t[2] for t in d["launches"] if t[0]=="list"]; print(sys.argv[2], "wall", round(d["wall_s"],3), "n_iter", d["n_iter"], "list", len(L), round(sum(L),1))'
for v in main G32 G16; do
  L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
  timeout -k 10 500 env ${L:+MW_LIB=$L} python -u tools/gpu/r5_c5fitdiag.py > "$OUT/diag_$v.json" 2> "$OUT/diag_$v.err" || { tail -5 "$OUT/diag_$v.err"; exit 1; }
  python -c "$summ" "$OUT/diag_$v.json" $v
done
echo "[listgb] done"
