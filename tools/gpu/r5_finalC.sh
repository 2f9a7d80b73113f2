#!/bin/bash
# Round-5 final tree, part C: the config-5 4-slide share (4 generator-sourced
# 40k^2 x 50 slides on one GPU) bench line.
set -o pipefail
TAG=${1:-r5finalC}
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py --slides-per-gpu 4 --size 40000 --channels 50 --source synth --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5x4.json" 2> "$OUT/bench_c5x4.err" || { tail -5 "$OUT/bench_c5x4.err"; exit 1; }
echo "[finalC] done"
