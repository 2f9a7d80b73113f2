#!/bin/bash
# Same-box A/B of the blur band width in the whole bench, and a per-launch
# trace of the batched k sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for bt in 8 4 8 4; do
  timeout -k 10 300 env MW_BLUR_BT=$bt python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_bt$bt.json 2> gpurun_out/ab/bench_bt$bt.err || { tail -3 gpurun_out/ab/bench_bt$bt.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('BT', sys.argv[2], 'bench ms', round(d['ms_per_step'],3), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()})" gpurun_out/ab/bench_bt$bt.json $bt
done
timeout -k 10 300 python tools/dev/sweep_trace.py 10000 gpurun_out/ab/sweep_trace.json > gpurun_out/ab/sweep_trace.log 2>&1 || { tail -3 gpurun_out/ab/sweep_trace.log; exit 1; }
echo "[gpu] done"
