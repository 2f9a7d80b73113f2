#!/bin/bash
# Round-4: QC sums as extra outputs of the label pass (label_tissue_regions(qc=True));
# the QC, stream and parity GPU tests (bitwise equalities across blur modes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qc}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 900 python -u -m pytest tests/test_gpu_qc.py tests/test_gpu_stream.py tests/test_gpu_parity.py -x -v --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
echo "[qc] done"
