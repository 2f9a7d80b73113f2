#!/bin/bash
# Round-4 GPU pass 5: defaults after the r4e A/B (kList as in round 3,
# kFirstSum at F > 32, dense pass opt-in) -- kinds exactness, config 2 / 5,
# design-point spreads, config-5 kernel statistics, SQ counters of the dense
# pass.
set -o pipefail
TAG=${1:-r4f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline"
B5="--size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lloyd_kinds.py -x -v --timeout 300 $T -m gpu > $OUT/kinds.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py $B > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 300 python -u bench.py $B5 > $OUT/c5.json 2> $OUT/c5.err || exit 1
for sp in 0.06 0.07 0.08 0.10; do
  MW_SYNTH_SPREAD=$sp timeout -k 10 200 python -u bench.py --mode design --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2_design_$sp.json 2> $OUT/c2_design_$sp.err || exit 1
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err" ) || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c2" -o c2 -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c2.json" 2> "$R/$OUT/prof_c2.err" ) || exit 1
# SQ counters of the dense pass (sweep, dense every pass)
P="$R/$OUT/pmc_dense"; mkdir -p "$P"
export MW_LLOYD_DENSE=1 MW_LLOYD_DENSE_MIN=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d "$P/sq1" -o run -- python "$R/bench.py" --sweep --steps 1 --warmup 0 --no-cpu-baseline > "$P/sq1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$P/sq2" -o run -- python "$R/bench.py" --sweep --steps 1 --warmup 0 --no-cpu-baseline > "$P/sq2.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d "$P/sq3" -o run -- python "$R/bench.py" --sweep --steps 1 --warmup 0 --no-cpu-baseline > "$P/sq3.log" 2>&1 || exit 1
echo "[pass5] done"
