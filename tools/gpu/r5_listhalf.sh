#!/bin/bash
# half-tile list pass: exactness tests, config-5 share fit history and config-2
# bench against the previous library (tools/probe/liblist_OLD.so), same box
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-listhalf}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
tail -1 "$OUT/kinds.log"
summ='import json,sys; d=json.load(open(sys.argv[1])); L=[t[2] for t in d["launches"] if t[0]=="list"]; print(sys.argv[2], "wall", round(d["wall_s"],3), "n_iter", d["n_iter"], "list", len(L), round(sum(L),1))'
for v in main OLD; do
  L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
  timeout -k 10 500 env ${L:+MW_LIB=$L} python -u tools/gpu/r5_c5fitdiag.py > "$OUT/diag_$v.json" 2> "$OUT/diag_$v.err" || { tail -5 "$OUT/diag_$v.err"; exit 1; }
  python -c "$summ" "$OUT/diag_$v.json" $v
done
bsum='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],2), {k:round(v["total_ms_per_step"],2) for k,v in d["kernels"].items() if k.startswith("lloyd") or k=="kmeans_fit"})'
for r in 1 2; do
  for v in main OLD; do
    L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
    timeout -k 10 300 env ${L:+MW_LIB=$L} MW_LLOYD_TRACE=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || { tail -3 "$OUT/c2_${v}_$r.err"; exit 1; }
    python -c "$bsum" "$OUT/c2_${v}_$r.json" "c2 $v"
  done
done
echo "[listhalf] done"
