#!/bin/bash
# per-kernel device times at MW_KBLOCKS 1024 / 768 (rocprofv3 kernel stats, config 2)
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-gridprof}"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
for g in 1024 768; do
  MW_KBLOCKS=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$g" -o c2 -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/b$g.json" 2> "$OUT/b$g.err" || { tail -3 "$OUT/b$g.err"; exit 1; }
done
cd "$R" && python - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
res = {}
for g in (1024, 768):
    f = glob.glob(f"{out}/p{g}/**/*kernel_stats.csv", recursive=True)[0]
    res[g] = {r["Name"][:70]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f))}
for n in sorted(res[1024], key=lambda n: -res[1024][n][0] * res[1024][n][1])[:22]:
    a = res[1024][n]; b = res[768].get(n, (0, 0))
    print(f"{n:70s} {a[0]:5d} {a[1]:9.1f} {b[1]:9.1f}")
PY
echo "[gridprof] done"
