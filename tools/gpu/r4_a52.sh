#!/bin/bash
# Round-4 A/B: the label pass at 33..52 channels on 26 feature pairs
# (assign_kernel<52, 64, true, true>) against the committed lib
# (abv/lib_head.so): parity / QC / stream GPU tests, config 5 x2 alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4a52}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_qc.py tests/test_gpu_stream.py -x -q --timeout 300 $T -m gpu > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_new$r.json 2> $OUT/c5_new$r.err || exit 1
  MW_LIB=abv/lib_head.so timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_head$r.json 2> $OUT/c5_head$r.err || exit 1
done
echo "[a52] done"
