#!/bin/bash
# Round-4 GPU pass: streaming tests, the whole GPU suite, the config-2 bench.
# usage: tools/gpu/r4_pass.sh TAG
set -o pipefail
TAG=${1:-r4a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 600 --timeout-method thread \
  -m gpu -k "not config5" > $OUT/stream.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
  --ignore tests/test_gpu_stream.py > $OUT/gpu.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 900 --timeout-method thread \
  -m gpu -k "config5" > $OUT/stream_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
