#!/bin/bash
# A/B of an environment toggle on the bench and the sweep bench:
#   gpurun -- 'AB="MW_LLOYD_XCD=0 MW_LLOYD_XCD=1" bash tools/dev/ab_env.sh'
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/abenv"
for kv in ${AB}; do
  echo "== $kv"
  if [ -z "$NOSWEEP" ]; then
    env "$kv" timeout -k 10 300 python "$R/tools/sweep_bench.py" --size 10000 --reps 1 > "$R/gpurun_out/abenv/sweep_$kv.json" 2> "$R/gpurun_out/abenv/sweep_$kv.err" || { tail -3 "$R/gpurun_out/abenv/sweep_$kv.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('sweep batched', round(d['batched']['s'],4), d['batched']['kernels_ms'], 'seq', round(d['sequential']['s'],4), 'same', d['identical_curve'])" "$R/gpurun_out/abenv/sweep_$kv.json"
  fi
  if [ -z "$NOBENCH" ]; then
    env "$kv" timeout -k 10 300 python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/abenv/bench_$kv.json" 2> "$R/gpurun_out/abenv/bench_$kv.err" || { tail -3 "$R/gpurun_out/abenv/bench_$kv.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench ms', round(d['ms_per_step'],3), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()})" "$R/gpurun_out/abenv/bench_$kv.json"
  fi
done
