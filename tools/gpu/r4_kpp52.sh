#!/bin/bash
# Round-4 A/B: k-means++ passes at 33 <= F <= 52 on the FMAX = 52 instances
# (default) against FMAX = 64 (MW_KPP_FM52=0), same library: kinds tests
# (incl. the FM52-vs-FM64 bitwise test), the config-5 full-size test, then the
# config-5 slice x2 alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r4fm52}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
T="--timeout-method thread"
timeout -k 10 700 python -u -m pytest tests/test_gpu_lloyd_kinds.py tests/test_gpu_fullsize.py -x -v --timeout 600 $T -m gpu -k "not config2" > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_fm52_$r.json 2> $OUT/c5_fm52_$r.err || exit 1
  MW_KPP_FM52=0 timeout -k 10 300 python -u bench.py --size 40000 --channels 50 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_fm64_$r.json 2> $OUT/c5_fm64_$r.err || exit 1
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o c5 -- python "$R/bench.py" --size 40000 --channels 50 --steps 1 --warmup 1 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err" ) || exit 1
echo "[fm52] done"
