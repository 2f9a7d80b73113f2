#!/bin/bash
# Round-4 GPU pass 3: pass-kind exactness (dense MFMA pass), the whole GPU
# suite (rank index, W2 first pass), config-2 A/B (rank index vs table,
# LDS-atomic first pass), sweep A/B (dense thresholds), config-5 slide.
set -o pipefail
TAG=${1:-r4d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline"
SW="--sweep --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu > $OUT/kinds.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests -x -v --timeout 900 $T -m gpu --deselect tests/test_gpu_lloyd_kinds.py > $OUT/gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > $OUT/c2_a.json 2> $OUT/c2_a.err && \
MW_RANK_TABLE=1 timeout -k 10 200 python -u bench.py $B > $OUT/c2_table.json 2> $OUT/c2_table.err && \
MW_LLOYD_FIRST_ATOMIC=1 timeout -k 10 200 python -u bench.py $B > $OUT/c2_fatomic.json 2> $OUT/c2_fatomic.err && \
timeout -k 10 200 python -u bench.py $B > $OUT/c2_b.json 2> $OUT/c2_b.err && \
timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d3.json 2> $OUT/sw_d3.err && \
MW_LLOYD_DENSE=0 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_nodense.json 2> $OUT/sw_nodense.err && \
MW_LLOYD_DENSE_MIN=1 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d1.json 2> $OUT/sw_d1.err && \
MW_LLOYD_DENSE_MIN=6 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d6.json 2> $OUT/sw_d6.err && \
timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_1.json 2> $OUT/c5_1.err
