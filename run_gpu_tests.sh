#!/bin/bash
# GPU pass: parity tests → sharded-fit check → bench → rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && (stop at
# the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
STEPS="${STEPS:-pytest,dist,bench,prof}"
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has pytest; then
  echo "[gpu] pytest -m gpu"; 
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if has dist; then
  echo "[gpu] 2-rank sharded fit check"
  timeout -k 10 300 torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tests/dist_gpu_check.py > gpurun_out/dist_check.log 2>&1
  rc=$?; grep -E "dist_gpu_check|Error|error" gpurun_out/dist_check.log | tail -5; [ $rc -eq 0 ] || { echo "dist rc=$rc"; exit $rc; }
fi
if has bench; then
  echo "[gpu] bench"
  timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
fi
if has prof; then
  echo "[gpu] rocprofv3 kernel trace"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err"
  rc=$?; cat "$R/gpurun_out/prof_bench.json"; [ $rc -eq 0 ] || { tail -20 "$R/gpurun_out/prof.err"; echo "prof rc=$rc"; exit $rc; }
  find "$R/gpurun_out/prof" -name "*stats*.csv" | head
fi
echo "[gpu] all done"
