#!/bin/bash
# Session-3 GPU pass: parity tests (incl. fused epilogues), HBM probe, bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
echo "[gpu] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
echo "[gpu] hbm probe"
timeout -k 10 120 ./tools/probe/hbm_probe > gpurun_out/hbm_probe.txt 2>&1 || exit 1
cat gpurun_out/hbm_probe.txt
echo "[gpu] bench"
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cut -c1-300 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
echo "[gpu] rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof6" -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof6_bench.json" 2> "$R/gpurun_out/prof6.err" || { tail -5 "$R/gpurun_out/prof6.err"; exit 1; }
echo "[gpu] done"
