#!/bin/bash
# Round-4: the LDS-atomic first-pass M-step (MW_LLOYD_FIRST_ATOMIC=1) against
# kFirstSum at config 5 (kernel times from rocprofv3), same call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4fa}; mkdir -p $OUT
R="$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for a in 0 1; do
  ( cd /tmp && export TMPDIR=/tmp && MW_LLOYD_FIRST_ATOMIC=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_a$a" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/c5_a$a.json" 2> "$R/$OUT/c5_a$a.err" ) || exit 1
done
echo "[fa] done"
