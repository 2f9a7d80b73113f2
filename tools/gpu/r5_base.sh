#!/bin/bash
# Round-5 baseline: config-2 bench lines for the materialised pipeline and the
# deferred-blur (non-materialised) pipeline, banded and fused label pass, each
# with a rocprofv3 kernel-stats pass.
set -o pipefail
TAG=${1:-r5base}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu-baseline --no-design-point --steps 10 --warmup 3"
timeout -k 10 200 $B > "$OUT/mat.json" 2> "$OUT/mat.err" || { tail -5 "$OUT/mat.err"; exit 1; }
MW_FUSED_BLUR=1 timeout -k 10 200 $B > "$OUT/def_band.json" 2> "$OUT/def_band.err" || { tail -5 "$OUT/def_band.err"; exit 1; }
MW_FUSED_BLUR=1 MW_DEFERRED_ASSIGN=fused timeout -k 10 200 $B > "$OUT/def_fused.json" 2> "$OUT/def_fused.err" || { tail -5 "$OUT/def_fused.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
P="python -u $R/bench.py --no-cpu-baseline --no-design-point --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o mat -- $P > "$OUT/prof_mat.log" 2>&1 || exit 1
MW_FUSED_BLUR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o defb -- $P > "$OUT/prof_defb.log" 2>&1 || exit 1
MW_FUSED_BLUR=1 MW_DEFERRED_ASSIGN=fused timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o deff -- $P > "$OUT/prof_deff.log" 2>&1 || exit 1
echo "[r5base] done"
