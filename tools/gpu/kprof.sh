#!/bin/bash
# rocprofv3 kernel stats of tools/kbench.py (ONLY=kpp,lloyd,...): per-kernel
# average durations into gpurun_out/kprof/<tag>_kernel_stats.csv
#   gpurun -- 'ONLY=kpp TAG=x bash tools/gpu/kprof.sh'
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/kprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kprof" -o "${TAG:-k}" -- \
  python "$R/tools/kbench.py" --only "${ONLY:-kpp}" --reps "${REPS:-5}" > "$R/gpurun_out/kprof/${TAG:-k}.txt" 2>&1 || exit 1
python - "$R/gpurun_out/kprof/${TAG:-k}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{int(r['Calls']):5d}  {r['Name'][:100]}")
PY
