#!/bin/bash
# SQ counter passes over blur_bench (one variant) for one library:
#   gpurun -- 'LIB=FAST ENVV="MW_BLUR_BT=8" bash tools/dev/blur_pmc.sh'
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/bpmc_${LIB:-base}"; mkdir -p "$OUT"
L="$R/milwrm_amd/libmilwrm_amd.so"; [ -n "$LIB" ] && L="$R/milwrm_amd/lib_$LIB.so"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  MW_LIB="$L" timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$R/tools/blur_bench.py" ${SIZE:-10000} 30 "${ENVV}" > "$OUT/$name.log" 2>&1 || { tail -3 "$OUT/$name.log"; exit 1; }
}
has() { [[ ",${PASSES:-sq1,sq2,sq3}," == *",$1,"* ]]; }
has sq1 && pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS
has sq2 && pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
has sq3 && pass sq3 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY
has ic && pass ic SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "blur" in r.get("Kernel_Name", ""):
            per[(f, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
acc = collections.defaultdict(list)
for (f, d, c), v in per.items():
    acc[c].append(v)
for k, v in sorted(acc.items()):
    print(f"{k:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
