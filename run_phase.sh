#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "[gpu] pytest"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "[gpu] phase timing"
timeout -k 10 600 python tools/phase_timing.py > gpurun_out/phase.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/phase.txt | tail -4; [ $rc -eq 0 ] || exit $rc
echo "[gpu] bench"
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cut -c1-400 gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
echo "[gpu] rocprof"
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof3" -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof3_bench.json" 2> "$R/gpurun_out/prof3.err" || exit 1
echo "[gpu] done"
