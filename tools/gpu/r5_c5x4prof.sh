#!/bin/bash
# config-5 share (4 synth slides per GPU): one step under a kernel trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-c5x4prof}"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c5 -- python3 -u "$R/bench.py" --no-cpu-baseline --steps 1 --warmup 0 --slides-per-gpu 4 --size 40000 --channels 50 --source synth > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
echo done
