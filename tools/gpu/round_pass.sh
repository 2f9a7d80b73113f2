#!/bin/bash
# GPU pass (STEPS=tests,bench,sweep,prof,pmc): parity tests (incl. the 2-rank sharded test), bench,
# k-sweep bench, rocprofv3 kernel stats, PMC HBM traffic passes; each step under its own limit.
#   gpurun -- bash tools/gpu/round_pass.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
STEPS="${STEPS:-tests,bench,sweep,prof,pmc}"
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  echo "[gpu] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
fi
if has bench; then
  echo "[gpu] bench"
  timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cut -c1-300 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
fi
if has sweep; then
  echo "[gpu] sweep bench"
  timeout -k 10 600 python tools/sweep_bench.py --size 10000 --reps 1 > gpurun_out/sweep.json 2> gpurun_out/sweep.err
  rc=$?; cut -c1-400 gpurun_out/sweep.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep.err; exit $rc; }
fi
if has prof; then
  echo "[gpu] rocprof"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err" ) || { tail -5 "$R/gpurun_out/prof.err"; exit 1; }
fi
if has pmc; then
  echo "[gpu] pmc"
  PMC_PASSES=fetch,write bash "$R/tools/gpu/pmc_bench.sh" || exit 1
fi
echo "[gpu] done"
