#!/bin/bash
# config-2 A/B of an env toggle ($AB_VAR), alternating runs, + one kernel trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${1:-abc2}"; mkdir -p "$OUT"; cd "$R" || exit 1
V=${AB_VAR:-MW_DRAWS_BESIDE}
for i in 1 2; do
  for v in 0 1; do
    env $V=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --no-design-point > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err" || { tail -5 "$OUT/b_${v}_$i.err"; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o tr -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 2 --no-design-point > "$OUT/prof.log" 2>&1 || exit 1
echo "[ab] done"
