#!/bin/bash
# Round-4 GPU pass 4: dense pass (XCD-aware groups, batched scans) exactness
# and sweep A/B; stream tests over rank table / index; config-2 default.
set -o pipefail
TAG=${1:-r4e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline"
SW="--sweep --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu > $OUT/kinds.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 300 $T -m gpu -k "not config5" > $OUT/stream.log 2>&1 && \
MW_LLOYD_DENSE_MIN=1 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d1.json 2> $OUT/sw_d1.err && \
MW_LLOYD_DENSE=0 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_nodense.json 2> $OUT/sw_nodense.err && \
timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d3.json 2> $OUT/sw_d3.err && \
timeout -k 10 200 python -u bench.py $B > $OUT/c2.json 2> $OUT/c2.err
