#!/bin/bash
# Round 6: timeline of the config-2 step (kernel + memory-copy trace, for the
# host gaps: tools/gap_report.py) and a host cProfile of the same bench.
set -o pipefail
TAG=${1:-r6trace}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/trace" -o c2 -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-design-point --no-host-outputs > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" ) || { tail -5 "$OUT/trace_bench.err"; exit 1; }
KT=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
MT=$(find "$OUT/trace" -name "*memory_copy_trace.csv" | head -1)
python tools/gap_report.py "$KT" $MT --last-ms 80 > "$OUT/gaps.txt" 2>&1 || true
tail -40 "$OUT/gaps.txt"
MW_BENCH_CPROFILE="$OUT/cprof" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-design-point > "$OUT/cprof_bench.json" 2> "$OUT/cprof_bench.err" || { tail -5 "$OUT/cprof_bench.err"; exit 1; }
python -c "
import pstats; p = pstats.Stats('$OUT/cprof.0'); p.sort_stats('cumulative').print_stats(60)" > "$OUT/cprof.txt" 2>&1
echo "[r6_trace] done"
