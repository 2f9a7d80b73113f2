#!/bin/bash
# Round-5 dense2 check: the pass-kinds exactness test at F = 30, then the
# sweep with the dense pass (MW_LLOYD_DENSE=1) and its kernel stats.
set -o pipefail
TAG=${1:-r5d2}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "30" > "$OUT/kinds.log" 2>&1 || { tail -30 "$OUT/kinds.log"; exit 1; }
B="python -u bench.py --sweep --no-cpu-baseline --steps 2 --warmup 1"
MW_LLOYD_DENSE=1 timeout -k 10 200 $B > "$OUT/sw_dense2.json" 2> "$OUT/sw_dense2.err" || { tail -5 "$OUT/sw_dense2.err"; exit 1; }
MW_LLOYD_DENSE=1 MW_LLOYD_DENSE_MIN=2 timeout -k 10 200 $B > "$OUT/sw_dense2_min2.json" 2> "$OUT/sw_dense2_min2.err" || { tail -5 "$OUT/sw_dense2_min2.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
P="python -u $R/bench.py --sweep --no-cpu-baseline --steps 1 --warmup 1"
MW_LLOYD_DENSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o dense2 -- $P > "$OUT/prof_d.log" 2>&1 || exit 1
echo "[r5d2] done"
