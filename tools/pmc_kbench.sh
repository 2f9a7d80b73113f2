#!/bin/bash
# PMC passes over tools/kbench.py (one pass per counter group):
#   TAG=x ONLY=lloyd1 [MW_LIB=...] bash tools/pmc_kbench.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc_${TAG:-kb}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$R/tools/kbench.py" --only "${ONLY:-lloyd1}" --reps 2 > "$OUT/$name.log" 2>&1
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit 1
pass sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
echo done
