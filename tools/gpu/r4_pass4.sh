#!/bin/bash
# Round-4 GPU pass 4: dense pass (XCD-aware groups, batched scans) exactness
# and sweep A/B; stream tests over rank table / index; k-means++ VGPR table
# and first-pass per-feature sums A/B (config 2 and 5); config-5 kernel stats.
set -o pipefail
TAG=${1:-r4e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline"
B5="--size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline"
SW="--sweep --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu > $OUT/kinds.log 2>&1 && \
MW_LLOYD_FIRST_SUM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu -k equal_full > $OUT/kinds_fsum.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 300 $T -m gpu -k "not config5" > $OUT/stream.log 2>&1 && \
MW_KPP_VTAB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 $T -m gpu -k "kpp or kmeans" > $OUT/kpp_vtab.log 2>&1 && \
MW_LLOYD_DENSE_MIN=1 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_d1.json 2> $OUT/sw_d1.err && \
MW_LLOYD_DENSE=0 timeout -k 10 300 python -u bench.py $SW > $OUT/sw_nodense.json 2> $OUT/sw_nodense.err && \
timeout -k 10 200 python -u bench.py $B > $OUT/c2.json 2> $OUT/c2.err && \
MW_KPP_VTAB=1 timeout -k 10 200 python -u bench.py $B > $OUT/c2_vtab.json 2> $OUT/c2_vtab.err && \
MW_LLOYD_FIRST_SUM=1 timeout -k 10 200 python -u bench.py $B > $OUT/c2_fsum.json 2> $OUT/c2_fsum.err && \
timeout -k 10 300 python -u bench.py $B5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
MW_LLOYD_FIRST_SUM=1 timeout -k 10 300 python -u bench.py $B5 > $OUT/c5_fsum.json 2> $OUT/c5_fsum.err || exit 1
for sp in 0.05 0.03 0.02; do
  MW_SYNTH_SPREAD=$sp timeout -k 10 200 python -u bench.py --mode design --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2_design_$sp.json 2> $OUT/c2_design_$sp.err || exit 1
done
