#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
echo "[gpu] host profile"
timeout -k 10 600 python tools/profile_step.py > gpurun_out/host_profile.txt 2>&1 || exit $?
head -3 gpurun_out/host_profile.txt
echo "[gpu] rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof2" -o bench -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof2_bench.json" 2> "$R/gpurun_out/prof2.err" || { tail -5 "$R/gpurun_out/prof2.err"; exit 1; }
echo "[gpu] done"
