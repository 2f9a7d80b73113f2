#!/bin/bash
# Same-box A/B of the main library against variant libraries (milwrm_amd/lib_<V>.so):
# GPU tests on the main library, then config-2 bench and config-5 slice runs
# alternating between the libraries.
#   VARIANTS="OLD" TESTS="tests/test_gpu_lloyd_kinds.py" C2=2 C5=1 bash tools/dev/ab_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_ab.log 2>&1
  rc=$?; tail -2 gpurun_out/ab/pytest_ab.log; grep -E "^FAILED|^ERROR" gpurun_out/ab/pytest_ab.log | head; [ $rc -eq 0 ] || exit $rc
fi
summ='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["ms_per_step"],2), {k:round(v["total_ms_per_step"],2) for k,v in d["kernels"].items()})'
for r in $(seq 1 ${C2:-0}); do
  for v in main $VARIANTS; do
    L=""; [ $v = main ] || L="$GRAFT_REPO_ROOT/milwrm_amd/lib_$v.so"
    timeout -k 10 300 env ${L:+MW_LIB=$L} MW_LLOYD_TRACE=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/c2_$v.json 2> gpurun_out/ab/c2_$v.err || { tail -3 gpurun_out/ab/c2_$v.err; exit 1; }
    python -c "$summ" gpurun_out/ab/c2_$v.json "c2 $v"
  done
done
for r in $(seq 1 ${C5:-0}); do
  for v in main $VARIANTS; do
    L=""; [ $v = main ] || L="$GRAFT_REPO_ROOT/milwrm_amd/lib_$v.so"
    timeout -k 10 400 env ${L:+MW_LIB=$L} MW_LLOYD_TRACE=1 python bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/c5_$v.json 2> gpurun_out/ab/c5_$v.err || { tail -3 gpurun_out/ab/c5_$v.err; exit 1; }
    python -c "$summ" gpurun_out/ab/c5_$v.json "c5 $v"
  done
done
# k sweep (tools/sweep_bench.py) on the main library under each SWEEP_ENVS entry
# ("-" = no extra env), alternating, SWEEP rounds
for r in $(seq 1 ${SWEEP:-0}); do
  for e in ${SWEEP_ENVS:--}; do
    E=""; [ "$e" = "-" ] || E="$e"
    timeout -k 10 300 env $E MW_NOOP=1 python tools/sweep_bench.py --size 10000 --reps 1 > gpurun_out/ab/sweep.json 2> gpurun_out/ab/sweep.err || { tail -3 gpurun_out/ab/sweep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('sweep', sys.argv[2], round(d['batched']['s'],4), d['batched'].get('kernels_ms'), 'same', d['identical_curve'])" gpurun_out/ab/sweep.json "$e"
  done
done
echo "[ab] done"
