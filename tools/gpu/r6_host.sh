#!/bin/bash
# Round 6: host timeline of the config-2 step (tools/dev/host_timeline.py)
set -o pipefail
TAG=${1:-r6host}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/dev/host_timeline.py --steps 3 > "$OUT/host_timeline.txt" 2>"$OUT/host_timeline.err" || { tail -5 "$OUT/host_timeline.err"; exit 1; }
tail -80 "$OUT/host_timeline.txt"
