#!/bin/bash
# Round-3 counters: PMC passes (SQ, MFMA busy, FETCH_SIZE, WRITE_SIZE) over one
# bench step at config 2 and at the config-5 slice, then rocprofv3 kernel
# stats of the config-5 slice.  Each pass under its own hard limit.
#   gpurun --timeout 1100 -- bash tools/gpu/r3_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$SKIP_C2" ]; then
  TAG=r3c2 PMC_PASSES="${C2_PASSES:-sq,mfma,fetch,write}" bash tools/gpu/pmc_bench.sh || exit 1
fi
if [ -z "$SKIP_C5" ]; then
  TAG=r3c5 BENCH_ARGS="--size 40000 --channels 50" PMC_PASSES="${C5_PASSES:-sq,mfma,fetch,write}" bash tools/gpu/pmc_bench.sh || exit 1
fi
if [ -n "$C5_PROF" ]; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c5" -o c5 -- python "$GRAFT_REPO_ROOT/bench.py" --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_c5.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_c5.err" ) || { tail -5 gpurun_out/prof_c5.err; exit 1; }
fi
echo "[pmc] all done"
