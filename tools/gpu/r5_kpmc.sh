#!/bin/bash
# SQ / SQC counter passes over $CMD, summarised per kernel matching $MATCH
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/kpmc_${TAG:-x}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $CMD > "$OUT/$name.log" 2>&1 || { tail -3 "$OUT/$name.log"; exit 1; }
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE
pass sqc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
python3 - "$OUT" "${MATCH}" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r.get("Kernel_Name", ""):
            per[r["Counter_Name"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:28s} {v:.4g}")
PY
echo "[kpmc] done"
