#!/bin/bash
# counter calibration of the deferred-blur sample path (tools/pmc_calib_r5.py)
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-calib5}"; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 200 python -u tools/pmc_calib_r5.py > "$OUT/calib.json" 2> "$OUT/calib.err" || { tail -5 "$OUT/calib.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/tools/pmc_calib_r5.py" > "$OUT/fetch.log" 2>&1 || { tail -3 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/tools/pmc_calib_r5.py" > "$OUT/write.log" 2>&1 || { tail -3 "$OUT/write.log"; exit 1; }
cd "$R" && python tools/pmc_calib_r5_report.py "$OUT" "$OUT/calib.json" "$OUT/table.json" > "$OUT/report.txt" 2>&1 || exit 1
echo "[calib] done"
