#!/bin/bash
# Round-4 GPU pass 7: SQ counters of the config-5 k-means++ and first Lloyd
# passes (one 40k^2 x 50 slide step), then the default bench (with its
# design-point line).
set -o pipefail
TAG=${1:-r4h}
OUT=gpurun_out/$TAG
R="$GRAFT_REPO_ROOT"
mkdir -p $OUT
P="$R/$OUT/pmc_c5"; mkdir -p "$P"
BA="--size 40000 --channels 50 --steps 1 --warmup 0 --no-cpu-baseline"
( cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d "$P/sq1" -o run -- python "$R/bench.py" $BA > "$P/sq1.log" 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$P/sq2" -o run -- python "$R/bench.py" $BA > "$P/sq2.log" 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d "$P/sq3" -o run -- python "$R/bench.py" $BA > "$P/sq3.log" 2>&1 || exit 1
) || exit 1
cd "$R" && timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
echo "[pass7] done"
