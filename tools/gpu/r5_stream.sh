#!/bin/bash
# Round-5: the config-5 shares (2 and 4 slides per GPU), the repeated
# config-5 label pass (band-buffer sizing), the stream tests, then the
# default bench line (host-output timing) and the 4-slide cohort line.
set -o pipefail
TAG=${1:-r5stream}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONUNBUFFERED=1
T="--timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 800 $T -m gpu --durations=0 > "$OUT/pytest_stream.log" 2>&1 || { tail -30 "$OUT/pytest_stream.log"; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-design-point > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --slides-per-gpu 4 --source synth --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5x4.json" 2> "$OUT/c5x4.err" || { tail -5 "$OUT/c5x4.err"; exit 1; }
echo "[r5stream] done"
