#!/bin/bash
# Round-4: gather counter calibration (tools/gather_calib.py): timings, then
# FETCH_SIZE and WRITE_SIZE passes over the same three draw patterns.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${1:-r4k}/calib"; mkdir -p "$OUT"
cd "$R" && timeout -k 10 120 python -u tools/gather_calib.py > "$OUT/times.json" 2> "$OUT/times.err" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python "$R/tools/gather_calib.py" > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python "$R/tools/gather_calib.py" > "$OUT/write.log" 2>&1 || exit 1
echo "[calib] done"
