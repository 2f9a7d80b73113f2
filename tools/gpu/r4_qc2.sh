#!/bin/bash
# Round-4: QC tests (bitwise/golden) + label-pass QC bench after the QC kernel change
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qc2}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_qc.py -x -v --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/qc_label_bench.py --size 10000 --channels 30 > $OUT/qc_c2.json 2> $OUT/qc_c2.err || exit 1
timeout -k 10 700 python -u tools/qc_label_bench.py --size 40000 --channels 50 --reps 2 > $OUT/qc_c5.json 2> $OUT/qc_c5.err || exit 1
echo "[qc2] done"
