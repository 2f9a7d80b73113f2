#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-cprof_c2}"; mkdir -p "$OUT"; cd "$R" || exit 1
MW_BENCH_CPROFILE="$OUT/c2.prof" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 2 --no-design-point > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -5 "$OUT/c2.err"; exit 1; }
python - "$OUT/c2.prof.0" > "$OUT/cprof_c2.txt" <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1]); p.sort_stats("tottime").print_stats(40)
p.sort_stats("cumulative").print_stats(60)
PY
echo done
