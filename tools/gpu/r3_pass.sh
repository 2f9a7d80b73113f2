#!/bin/bash
# Round-3 GPU pass: parity tests (no -x: every failure is reported), smoke,
# bench, --gpus 2 must fail loudly on a one-GPU box, rocprof kernel stats.
# Each GPU step runs under its own limit; a crash/timeout ends the script.
#   gpurun --timeout 1200 -- bash tools/gpu/r3_pass.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
STEPS="${STEPS:-tests,smoke,bench,gpus2,prof}"
TESTS="${TESTS:-tests}"
has() { [[ ",$STEPS," == *",$1,"* ]]; }
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if has tests; then
  echo "[gpu] pytest -m gpu $TESTS"
  timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_gpu.log
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
  fatal $rc && exit $rc
fi
if has smoke; then
  echo "[gpu] smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  echo "[gpu] bench"
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cut -c1-400 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
fi
if has gpus2; then
  echo "[gpu] bench --gpus 2 on one GPU must fail"
  timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 > gpurun_out/gpus2.out 2>&1
  rc=$?; echo "rc=$rc"; tail -2 gpurun_out/gpus2.out
  fatal $rc && exit $rc
fi
if has prof; then
  echo "[gpu] rocprof"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err" ) || { tail -5 "$R/gpurun_out/prof.err"; exit 1; }
fi
echo "[gpu] done"
