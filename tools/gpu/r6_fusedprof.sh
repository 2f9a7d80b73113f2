#!/bin/bash
# Round 6: the deferred-blur config-2 step with the fused label epilogue
# (MW_FUSED_BLUR=1 MW_DEFERRED_ASSIGN=fused): kernel stats and SQ / MFMA
# counter passes of blur_mfma_kernel<..., 2> (kEpiAssign) and <..., 1> (kEpiSample)
set -o pipefail
TAG=${1:-r6fused}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
export MW_FUSED_BLUR=1 MW_DEFERRED_ASSIGN=fused
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" ) || { tail -5 "$OUT/bench_prof.err"; exit 1; }
TAG=${TAG}_c2 BENCH_ARGS="--no-design-point --no-host-outputs" PMC_PASSES=sq,sq2,mfma bash "$R/tools/gpu/pmc_bench.sh" > "$OUT/pmc.log" 2>&1 || { tail -5 "$OUT/pmc.log"; exit 1; }
python - "$OUT" "$R/gpurun_out/pmc_${TAG}_c2" <<'PY'
import csv, glob, sys, collections, json
out, base = sys.argv[1], sys.argv[2]
f = glob.glob(out + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r["Percentage"]) > 1.0:
        print(f"{r['Name'][:70]:70s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
for pas in ("sq", "sq2", "mfma"):
    per = collections.defaultdict(float)
    for g in glob.glob(f"{base}/{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(g)):
            n = r["Kernel_Name"]
            for key, pat in (("assign_epi", "true, 2>("), ("sample_epi", "true, 1>(")):
                if pat in n:
                    per[(key, r["Counter_Name"])] += float(r["Counter_Value"])
    for key in ("assign_epi", "sample_epi"):
        d = {c: v for (k, c), v in per.items() if k == key}
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        print(pas, key, {c: (round(v / wc, 3) if c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else "%.3g" % v) for c, v in sorted(d.items())})
PY
echo "[r6_fusedprof] done"
