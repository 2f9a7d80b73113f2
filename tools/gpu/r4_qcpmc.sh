#!/bin/bash
# Round-4: SQ counters of the QC kernel (tools/qc_label_bench.py, config 2 slide)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qcpmc}; mkdir -p $OUT
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d "$R/$OUT/sq" -o run -- python3 "$R/tools/qc_label_bench.py" --size 10000 --channels 30 --reps 1 > "$R/$OUT/sq.log" 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$R/$OUT/sq2" -o run -- python3 "$R/tools/qc_label_bench.py" --size 10000 --channels 30 --reps 1 > "$R/$OUT/sq2.log" 2>&1 || exit 1
echo "[qcpmc] done"
