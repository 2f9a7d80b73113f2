#!/bin/bash
# host-call costs and a config-2 bench after the allocator-statistics change
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4n}; mkdir -p $OUT
timeout -k 10 120 python -u tools/host_calls.py > $OUT/host_calls.json 2> $OUT/host_calls.err || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2b.json 2> $OUT/c2b.err || exit 1
echo "[host] done"
