#!/bin/bash
# rocprofv3 kernel averages of tools/kbench.py under each variant library
# milwrm_amd/lib_<V>.so (built with MW_EXTRA_FLAGS=-DMW_..._<V>), plus the
# default library:  gpurun -- 'VARIANTS="A B" ONLY=kpp bash tools/gpu/kvariants.sh'
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/kvar"
cd /tmp && export TMPDIR=/tmp
for v in base ${VARIANTS}; do
  lib="$R/milwrm_amd/libmilwrm_amd.so"; [ "$v" = base ] || lib="$R/milwrm_amd/lib_$v.so"
  echo "== $v"
  MW_LIB="$lib" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kvar" -o "$v" -- \
    python "$R/tools/kbench.py" --only "${ONLY:-kpp}" --reps "${REPS:-5}" > "$R/gpurun_out/kvar/$v.txt" 2>&1 || { tail -3 "$R/gpurun_out/kvar/$v.txt"; exit 1; }
  python - "$R/gpurun_out/kvar/${v}_kernel_stats.csv" "${MATCH:-kpp|lloyd|assign|gather|blur}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if re.search(sys.argv[2], r["Name"]):
        print(f"{float(r['AverageNs'])/1e3:9.1f} us x{int(r['Calls']):5d}  {r['Name'][:90]}")
PY
done
