#!/bin/bash
# Round 6: the other BASELINE shapes on the round-6 tree: the k = 2..20 sweep
# (config 4's per-GPU rows) and the config-5 4-slide share (one step; 40k^2 x
# 50 slides generated band by band), each under its own limit.
set -o pipefail
TAG=${1:-r6cfg}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --sweep --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/sweep.json" 2> "$OUT/sweep.err" || { tail -5 "$OUT/sweep.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/sweep.json')); s=d['sweep']; print('sweep', s['seconds'], s['best_k'], s.get('alu_roofline'))"
timeout -k 10 900 python -u bench.py --no-cpu-baseline --no-host-outputs --steps 1 --warmup 0 --slides-per-gpu 4 --size 40000 --channels 50 --source synth > "$OUT/c5x4.json" 2> "$OUT/c5x4.err" || { tail -5 "$OUT/c5x4.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/c5x4.json')); print('c5x4', d['ms_per_step'], {k: v['mean_ms'] for k, v in d['kernels'].items()}, d.get('pipeline_roofline'))"
echo "[r6_configs] done"
