#!/bin/bash
# HBM read ceiling at the step's stream sizes (tools/probe/hbm_probe2.hip)
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-r6probe}"; mkdir -p "$OUT"; cd "$R" || exit 1
for a in "2.2 1" "2.2 0" "6 1" "18 1"; do
  timeout -k 10 60 tools/probe/bin/hbm_probe2 $a >> "$OUT/hbm_probe2.txt" 2>&1 || exit 1
done
cat "$OUT/hbm_probe2.txt"
