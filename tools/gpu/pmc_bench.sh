#!/bin/bash
# PMC counter passes over one bench step (rocprofv3 --pmc, one pass per counter
# group, no tracing domains); each pass under its own hard time limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG="${TAG:-bench}"
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name="$1"; shift
  echo "[pmc] pass $name: $*"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$name.log" 2>&1
}
PASSES="${PMC_PASSES:-sq,sq2,fetch,write}"
has() { [[ ",$PASSES," == *",$1,"* ]]; }
if has sq; then pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS || exit 1; fi
if has sq2; then pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1; fi
if has mfma; then pass mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE || exit 1; fi
if has fetch; then pass fetch FETCH_SIZE || exit 1; fi
if has write; then pass write WRITE_SIZE || exit 1; fi
echo "[pmc] done"
