#!/bin/bash
# host profile of the timed sweep step (MW_BENCH_CPROFILE), dense passes on/off
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-cprof}"; mkdir -p "$OUT"; cd "$R" || exit 1
for d in 1 0; do
  MW_LLOYD_DENSE=$d MW_BENCH_CPROFILE="$OUT/sweep_d$d.prof" timeout -k 10 200 python -u bench.py --sweep --no-cpu-baseline --steps 1 --warmup 1 > "$OUT/sw_d$d.json" 2> "$OUT/sw_d$d.err" || { tail -5 "$OUT/sw_d$d.err"; exit 1; }
  python - "$OUT/sweep_d$d.prof.0" > "$OUT/cprof_d$d.txt" <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1]); p.sort_stats("tottime").print_stats(35)
p.sort_stats("cumulative").print_stats(45)
PY
done
echo done
MW_LLOYD_DENSE=1 timeout -k 10 200 python -u tools/gpu/r5_d2diag.py > "$OUT/d2diag.json" 2> "$OUT/d2diag.err" || { tail -5 "$OUT/d2diag.err"; exit 1; }
echo diag-done
