#!/bin/bash
# Round-4 A/B: the QC kernel's per-domain sums in registers (k <= 8, default)
# against the LDS form (MW_QC_REG=0): QC tests, then the label-pass QC bench
# at config 2 and config 5 with either.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qcreg}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 600 python -u -m pytest tests/test_gpu_qc.py -x -q --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
for r in 1 0; do
  MW_QC_REG=$r timeout -k 10 300 python -u tools/qc_label_bench.py --size 10000 --channels 30 > $OUT/qc_c2_reg$r.json 2> $OUT/qc_c2_reg$r.err || exit 1
done
for r in 1 0; do
  MW_QC_REG=$r timeout -k 10 600 python -u tools/qc_label_bench.py --size 40000 --channels 50 --reps 2 > $OUT/qc_c5_reg$r.json 2> $OUT/qc_c5_reg$r.err || exit 1
done
echo "[qcreg] done"
