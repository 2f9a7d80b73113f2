#!/bin/bash
# Lloyd-pass ablation: kbench lloyd0/lloyd1 per library variant (build_abl/lib_*.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-base a1 a2 a1w3}; do
  echo "== $v"
  MW_LIB="$GRAFT_REPO_ROOT/build_abl/lib_$v.so" timeout -k 10 120 python tools/kbench.py --only lloyd0,lloyd1,assign --reps 10 > gpurun_out/abl_$v.log 2>&1 || { tail -5 gpurun_out/abl_$v.log; exit 1; }
  grep -E "lloyd|kpp" gpurun_out/abl_$v.log
done
