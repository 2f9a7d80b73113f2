#!/bin/bash
# dense2 / fits-driver round: exactness tests, default sweep, SQ counters of the dense kernel
set -o pipefail
TAGN=${1:-d2all}
bash "$GRAFT_REPO_ROOT/tools/gpu/r5_d2t.sh" "$TAGN" || exit 1
export TAG="$TAGN" MATCH=lloyd_dense2 CMD="python -u $GRAFT_REPO_ROOT/bench.py --sweep --no-cpu-baseline --steps 1 --warmup 0"
bash "$GRAFT_REPO_ROOT/tools/gpu/r5_kpmc.sh" > "$GRAFT_REPO_ROOT/gpurun_out/$TAGN/kpmc.txt" 2>&1 || exit 1
echo "[d2all] done"
