#!/bin/bash
# k-means block-grid A/B (MW_KBLOCKS) at config 2: per-pass-kind device times
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-grid}"; mkdir -p "$OUT"; cd "$R" || exit 1
bsum='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],2), {k:round(v["total_ms_per_step"],3) for k,v in d["kernels"].items() if k.startswith("lloyd") or k.startswith("kpp") or k=="kmeans_fit"})'
for r in 1 2; do
  for g in 1024 768 512; do
    MW_KBLOCKS=$g MW_LLOYD_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/g${g}_$r.json" 2> "$OUT/g${g}_$r.err" || { tail -3 "$OUT/g${g}_$r.err"; exit 1; }
    python -c "$bsum" "$OUT/g${g}_$r.json" "G=$g"
  done
done
echo "[grid] done"
