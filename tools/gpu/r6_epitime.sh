#!/bin/bash
# Round 6: the deferred config-2 step's label pass, fused vs banded (kernel stats)
set -o pipefail
TAG=${1:-r6epit}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
for how in ${HOWS:-fused band}; do
  ( cd /tmp && export TMPDIR=/tmp && MW_FUSED_BLUR=1 MW_DEFERRED_ASSIGN=$how timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$how" -o c2 -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_$how.json" 2> "$OUT/bench_$how.err" ) || { tail -5 "$OUT/bench_$how.err"; exit 1; }
  python - "$OUT" "$how" <<'PY'
import csv, glob, json, sys
out, how = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/bench_{how}.json"))
print(how, round(d["ms_per_step"], 3), {k: v["mean_ms"] for k, v in d["kernels"].items()})
f = glob.glob(f"{out}/prof_{how}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "blur_mfma" in r["Name"] or "assign" in r["Name"]:
        print(f"   {r['Name'][:70]:70s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
echo "[r6_epitime] done"
