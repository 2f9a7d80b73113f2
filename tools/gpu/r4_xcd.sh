#!/bin/bash
# Round-4 A/B: the blur's XCD-grouped tile order (MW_BLUR_XCD=1: adjacent column
# bands on one XCD, halo columns shared in its L2) against the default, config 2,
# alternating, plus a FETCH_SIZE pass of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4xcd}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for x in 0 1; do
    MW_BLUR_XCD=$x timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-design-point > $OUT/c2_x${x}_$r.json 2> $OUT/c2_x${x}_$r.err || exit 1
  done
done
R="$GRAFT_REPO_ROOT"
for x in 0 1; do
  ( cd /tmp && export TMPDIR=/tmp && MW_BLUR_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$OUT/pmc_x$x" -o p -- python "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-design-point > "$R/$OUT/pmc_x$x.json" 2> "$R/$OUT/pmc_x$x.err" ) || exit 1
done
echo "[xcd] done"
