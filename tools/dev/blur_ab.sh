#!/bin/bash
# A/B of blur variant libraries (tools/dev/build_variant.sh) on the GPU box:
#   gpurun -- 'LIBS="ACC FAST" VARS="|MW_BLUR_BT=8" bash tools/dev/blur_ab.sh'
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/ab"
VARS="${VARS:-}"
for v in ${LIBS}; do
  echo "== $v"
  MW_LIB="$R/milwrm_amd/lib_$v.so" BLUR_SAVE="$R/gpurun_out/ab/$v.npy" timeout -k 10 180 \
    python "$R/tools/blur_bench.py" ${SIZE:-10000} ${CH:-30} "${VARS//|/,}" || exit 1
done
python - $LIBS <<'PY'
import sys, numpy as np, os
R = os.environ["GRAFT_REPO_ROOT"]
a = {v: np.load(f"{R}/gpurun_out/ab/{v}.npy") for v in sys.argv[1:]}
base = sys.argv[1]
for v, x in a.items():
    d = np.abs(x - a[base]); print(f"{v} vs {base}: max abs {d.max():.3e}, max rel {(d / np.maximum(np.abs(a[base]), 1e-3)).max():.3e}")
PY
