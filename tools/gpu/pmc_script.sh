#!/bin/bash
# PMC counter passes (rocprofv3 --pmc, one pass per counter group, no tracing
# domains) for a python command: bash tools/gpu/pmc_script.sh <tag> <script.py> [args...]
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG="$1"; shift
SCRIPT="$R/$1"; shift
mkdir -p "$R/gpurun_out/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  echo "[pmc] pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/pmc_$TAG/$name" -o run -- python3 "$SCRIPT" "${ARGS[@]}" > "$R/gpurun_out/pmc_$TAG/$name.log" 2>&1
}
ARGS=("$@")
SQ="${PMC_SQ:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS}"
PASSES="${PMC_PASSES:-sq,fetch,write}"
has() { [[ ",$PASSES," == *",$1,"* ]]; }
if has sq; then pass sq $SQ || exit 1; fi
if has sq2; then pass sq2 ${PMC_SQ2:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_BUSY_CYCLES SQ_WAVES} || exit 1; fi
if has fetch; then pass fetch FETCH_SIZE || exit 1; fi
if has write; then pass write WRITE_SIZE || exit 1; fi
find "$R/gpurun_out/pmc_$TAG" -name "*counter_collection.csv" | head
echo "[pmc] done"
