#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4p}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 250 $T -m gpu -k slide_order > $OUT/sort_test.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_config34.py -x -v -s --timeout 900 $T -m gpu > $OUT/config34.log 2>&1 || exit 1
echo "[sort2] done"
