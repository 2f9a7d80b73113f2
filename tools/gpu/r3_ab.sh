#!/bin/bash
# Round-3 A/B pass: blur variant libraries (tools/dev/build_variant.sh), the
# bench with the blurred slide materialised vs deferred into the fused
# epilogues, and selected parity tests.  Each GPU step under its own limit.
#   gpurun --timeout 900 -- 'LIBS="OLD H16" TESTS="tests/test_gpu_parity.py" bash tools/gpu/r3_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ -n "$LIBS" ]; then
  echo "[gpu] blur A/B: $LIBS"
  timeout -k 10 400 env LIBS="$LIBS" SIZE="${SIZE:-10000}" CH="${CH:-30}" bash tools/dev/blur_ab.sh > gpurun_out/ab/blur_ab.log 2>&1
  rc=$?; cat gpurun_out/ab/blur_ab.log | grep -v "^$" | tail -12; fatal $rc && exit $rc
fi
if [ -n "$BH" ]; then
  echo "[gpu] blur band-height sweep: $BH"
  timeout -k 10 300 python tools/blur_bench.py ${SIZE:-10000} ${CH:-30} "$BH" > gpurun_out/ab/bh.log 2>&1
  rc=$?; grep "BW=" gpurun_out/ab/bh.log; fatal $rc && exit $rc
fi
if [ -n "$TESTS" ]; then
  echo "[gpu] pytest -m gpu $TESTS"
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/pytest.log; grep -E "^FAILED|^ERROR" gpurun_out/ab/pytest.log | head -20
  fatal $rc && exit $rc
fi
for mode in ${BENCH_MODES:-}; do
  echo "[gpu] bench MW_FUSED_BLUR=$mode"
  timeout -k 10 300 env MW_FUSED_BLUR=$mode python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_fused$mode.json 2> gpurun_out/ab/bench_fused$mode.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/bench_fused$mode.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench ms', round(d['ms_per_step'],3), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()}, d['roofline']['kernel'], round(d['roofline']['frac'],3))" gpurun_out/ab/bench_fused$mode.json
done
for da in ${C5_MODES:-}; do
  echo "[gpu] config-5 slice (40k^2 x 50) MW_DEFERRED_ASSIGN=$da"
  timeout -k 10 400 env MW_DEFERRED_ASSIGN=$da python bench.py --size 40000 --channels 50 --steps ${C5_STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_c5_$da.json 2> gpurun_out/ab/bench_c5_$da.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab/bench_c5_$da.err; exit $rc; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5 ms', round(d['ms_per_step'],1), {k:v['total_ms_per_step'] for k,v in d['kernels'].items()}, d['roofline']['kernel'], round(d['roofline']['frac'],3))" gpurun_out/ab/bench_c5_$da.json
done
if [ -n "$PROF" ]; then
  echo "[gpu] rocprof bench MW_FUSED_BLUR=$PROF"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 env MW_FUSED_BLUR=$PROF rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/ab/prof" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/ab/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/ab/prof.err" ) || { tail -5 gpurun_out/ab/prof.err; exit 1; }
  head -12 gpurun_out/ab/prof/bench_kernel_stats.csv | cut -c1-160
fi
echo "[gpu] done"
