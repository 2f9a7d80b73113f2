#!/bin/bash
# Round-4 SQ counters per kernel over short config-2 / config-5 bench runs
# (tools/dev/kern_pmc.sh passes: issue/wait breakdown, instruction mix, LDS,
# MFMA busy), each pass under its own hard limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
run() {  # TAG CMD
  local tag="$1"; shift
  local OUT="$R/gpurun_out/kpmc_$tag"; mkdir -p "$OUT"
  ( cd /tmp && export TMPDIR=/tmp
    for p in "sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS" \
             "sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
             "sq3 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
      set -- $p; name=$1; shift
      timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python "$R/bench.py" $BARGS > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -3 "$OUT/$name.log"; exit 1; }
    done ) || exit 1
  python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        per[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id"))
for (k, c), v in sorted(per.items()):
    print(f"{k:70s} {c:26s} {v:.6g} n={len(disp[(k, c)])}")
PY
}
BARGS="--steps 1 --warmup 0 --no-cpu-baseline" run c2 && \
BARGS="--size 40000 --channels 50 --steps 1 --warmup 0 --no-cpu-baseline" run c5
echo "[pmc] done"
