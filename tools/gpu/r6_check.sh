#!/bin/bash
# Round 6: a kernel change's same-bits check (fit fingerprint vs the recorded
# one), the named GPU tests, then kernel stats over the bench (rocprofv3).
#   r6_check.sh TAG "EXPECTED_FP_LINE_SUBSTRING" "pytest -k expression"
set -o pipefail
TAG=${1:-r6check}
EXP=${2:-}
KEXPR=${3:-}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/dev/fit_fingerprint.py > "$OUT/fp.txt" 2>&1 || { tail -5 "$OUT/fp.txt"; exit 1; }
grep FP "$OUT/fp.txt"
if [ -n "$EXP" ]; then grep -q "$EXP" "$OUT/fp.txt" && echo "FINGERPRINT SAME" || echo "FINGERPRINT DIFFERS"; fi
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "$KEXPR" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" ) || { tail -5 "$OUT/bench_prof.err"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
d = json.load(open(out + "/bench.json"))
print("bench", round(d["ms_per_step"], 3), {k: v["mean_ms"] for k, v in d["kernels"].items()})
f = glob.glob(out + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r["Percentage"]) > 0.5:
        print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
echo "[r6_check] done"
