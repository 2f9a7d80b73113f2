#!/bin/bash
# Round-5 sweep baseline: bench.py --sweep (k = 2..20 over config 2's rows)
# with the bounded passes and with the dense pass, plus rocprof stats of each.
set -o pipefail
TAG=${1:-r5sweep}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
B="python -u bench.py --sweep --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 200 $B > "$OUT/sw_bounded.json" 2> "$OUT/sw_bounded.err" || { tail -5 "$OUT/sw_bounded.err"; exit 1; }
MW_LLOYD_DENSE=1 timeout -k 10 200 $B > "$OUT/sw_dense.json" 2> "$OUT/sw_dense.err" || { tail -5 "$OUT/sw_dense.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
P="python -u $R/bench.py --sweep --no-cpu-baseline --steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bounded -- $P > "$OUT/prof_b.log" 2>&1 || exit 1
MW_LLOYD_DENSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o dense -- $P > "$OUT/prof_d.log" 2>&1 || exit 1
echo "[r5sweep] done"
