#!/bin/bash
# Same-box A/B of the library against a variant build (default lib_nont.so:
# MW_STREAM_NT=0): kernel stats of the config-2 bench, twice each,
# alternating; then the step time of each; with FP=1 first the variant's fit
# fingerprint.  "nt" = the default library, "nont" = the variant.
#   r6_nt_ab.sh TAG [VARIANT_LIB]
# The variant is built here first, e.g. MW_BUILD_DIR=build_nont
# MW_LIB=milwrm_amd/lib_nont.so MW_EXTRA_FLAGS=-DMW_STREAM_NT=0 python -m
# milwrm_amd.build, and must travel (.gpurunignore lists milwrm_amd/lib_*.so:
# narrow that pattern while the A/B runs).
set -o pipefail
TAG=${1:-r6ntab}
VLIB=${2:-lib_nont.so}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
if [ "${FP:-0}" = 1 ]; then
  MW_LIB="$R/milwrm_amd/$VLIB" timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp_variant.txt" 2>&1 || { tail -5 "$OUT/fp_variant.txt"; exit 1; }
  grep FP "$OUT/fp_variant.txt"
fi
for rep in 1 2; do
  for v in nt nont; do
    if [ "$v" = nont ]; then export MW_LIB="$R/milwrm_amd/$VLIB"; else unset MW_LIB; fi
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${v}_$rep" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof_${v}_$rep.json" 2> "$OUT/bench_prof_${v}_$rep.err" ) || { tail -5 "$OUT/bench_prof_${v}_$rep.err"; exit 1; }
  done
done
for rep in 1 2; do
  for v in nt nont; do
    if [ "$v" = nont ]; then export MW_LIB="$R/milwrm_amd/$VLIB"; else unset MW_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || { tail -5 "$OUT/bench_${v}_$rep.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${v}_$rep.json')); print('$v', $rep, round(d['ms_per_step'], 3))"
  done
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
t = collections.defaultdict(dict)
for v in ("nt", "nont"):
    for rep in (1, 2):
        f = glob.glob(f"{out}/prof_{v}_{rep}/**/*kernel_stats.csv", recursive=True)[0]
        for r in csv.DictReader(open(f)):
            t[r["Name"][:60]][f"{v}{rep}"] = float(r["AverageNs"]) / 1e3
for k, d in sorted(t.items(), key=lambda x: -x[1].get("nont1", 0)):
    if d.get("nont1", 0) > 50:
        print(f"{k:60s} " + " ".join(f"{c}={d.get(c, 0):8.1f}" for c in ("nt1", "nont1", "nt2", "nont2")))
PY
echo "[r6_nt_ab] done"
