#!/bin/bash
# Round-4: fused-epilogue bitwise test with the 50 / 45-channel cases and the
# 50-channel end-to-end oracle tests (52-channel label kernel, FMAX = 52 Lloyd)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4f50}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v --timeout 600 $T -m gpu -k "fused_epilogues or 50" > $OUT/tests.log 2>&1 || exit 1
echo "[f50] done"
