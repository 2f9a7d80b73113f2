#!/bin/bash
# Lloyd grid of 768 blocks at F <= 32: GPU tests, config-2 bench and sweep
# against the previous library (tools/probe/liblist_OLD.so), same box
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-gridval}"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bsum='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],2), {k:round(v["total_ms_per_step"],2) for k,v in d["kernels"].items() if k in ("kmeans_fit","assign_conf")})'
for r in 1 2; do
  for v in main OLD; do
    L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
    timeout -k 10 300 env ${L:+MW_LIB=$L} python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || { tail -3 "$OUT/c2_${v}_$r.err"; exit 1; }
    python -c "$bsum" "$OUT/c2_${v}_$r.json" "c2 $v"
  done
done
ssum='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],1))'
for v in main OLD; do
  L=""; [ $v = main ] || L="$R/tools/probe/liblist_$v.so"
  timeout -k 10 300 env ${L:+MW_LIB=$L} python -u bench.py --sweep --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/sw_$v.json" 2> "$OUT/sw_$v.err" || { tail -3 "$OUT/sw_$v.err"; exit 1; }
  python -c "$ssum" "$OUT/sw_$v.json" "sweep $v"
done
echo "[gridval] done"
