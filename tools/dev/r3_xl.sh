#!/bin/bash
# A/B of the label pass's LDS-row form (MW_ASSIGN_XL) on the bench at config 2
# and the config-5 slice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for xl in 1 0; do
  timeout -k 10 300 env MW_ASSIGN_XL=$xl python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_xl$xl.json 2> gpurun_out/ab/bench_xl$xl.err || { tail -3 gpurun_out/ab/bench_xl$xl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('XL', sys.argv[2], 'bench ms', round(d['ms_per_step'],3), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()}, round(d['roofline']['frac'],3))" gpurun_out/ab/bench_xl$xl.json $xl
done
for xl in 1 0; do
  timeout -k 10 400 env MW_ASSIGN_XL=$xl python bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c5_xl$xl.json 2> gpurun_out/ab/c5_xl$xl.err || { tail -3 gpurun_out/ab/c5_xl$xl.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('XL', sys.argv[2], 'c5 ms', round(d['ms_per_step'],1), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()})" gpurun_out/ab/c5_xl$xl.json $xl
done
