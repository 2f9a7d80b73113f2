#!/bin/bash
# Same-box A/B of the Lloyd full-E-step form (main library vs lib_NOXL: the
# round-2 kernel) on the bench and the k sweep, after the Lloyd exactness tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_lloyd.log 2>&1
rc=$?; tail -2 gpurun_out/ab/pytest_lloyd.log; [ $rc -eq 0 ] || exit $rc
for v in main NOXL main NOXL; do
  L=""; [ $v = NOXL ] && L="$GRAFT_REPO_ROOT/milwrm_amd/lib_NOXL.so"
  timeout -k 10 300 env ${L:+MW_LIB=$L} python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || { tail -3 gpurun_out/ab/bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'bench ms', round(d['ms_per_step'],3), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()})" gpurun_out/ab/bench_$v.json $v
done
for v in main NOXL; do
  L=""; [ $v = NOXL ] && L="$GRAFT_REPO_ROOT/milwrm_amd/lib_NOXL.so"
  timeout -k 10 300 env ${L:+MW_LIB=$L} python tools/sweep_bench.py --size 10000 --reps 1 > gpurun_out/ab/sweep_$v.json 2> gpurun_out/ab/sweep_$v.err || { tail -3 gpurun_out/ab/sweep_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'sweep', round(d['batched']['s'],4), d['batched']['kernels_ms'], 'same', d['identical_curve'])" gpurun_out/ab/sweep_$v.json $v
done
