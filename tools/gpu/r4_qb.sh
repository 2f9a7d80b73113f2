#!/bin/bash
# Round-4: kTile -> kList switch point (MW_LLOYD_QUEUE_BELOW) at config 2,
# headline (I = 5) and design point (I = 17), plus the sweep at 0.3 / 0.5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4qb}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for q in 0.2 0.1 0.3 0.2; do
  MW_LLOYD_QUEUE_BELOW=$q timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/c2_q$q.json 2> $OUT/c2_q$q.err || exit 1
done
for q in 0.2; do
  MW_LLOYD_QUEUE_BELOW=$q timeout -k 10 300 python -u bench.py --sweep --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sw_q$q.json 2> $OUT/sw_q$q.err || exit 1
done
echo "[qb] done"
