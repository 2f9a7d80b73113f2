#!/bin/bash
# Same-box A/B of the Lloyd full-E-step form on the config-5 slice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for v in main NOXL main NOXL; do
  L=""; [ $v = NOXL ] && L="$GRAFT_REPO_ROOT/milwrm_amd/lib_NOXL.so"
  timeout -k 10 400 env ${L:+MW_LIB=$L} MW_LLOYD_TRACE=1 python bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c5_$v.json 2> gpurun_out/ab/c5_$v.err || { tail -3 gpurun_out/ab/c5_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'c5 ms', round(d['ms_per_step'],1), 'fit', d['kernels']['kmeans_fit']['total_ms_per_step'])" gpurun_out/ab/c5_$v.json $v
done
