#!/bin/bash
# Dev variant of the library with one source rebuilt under extra flags (FILE,
# default blur_u16.hip); every other object is reused from build/.  The
# ablation / development macros (MW_ABL_*, MW_BLUR_DEV / _D / _F32H / _BT8,
# MW_COL_STATS_LDS) were taken out of the product kernels in round 4: a variant
# now carries its own patched source (git history holds the round-3 forms).
#   [FILE=lloyd.hip] bash tools/dev/build_variant.sh NAME [-DFLAG ...]  ->  milwrm_amd/lib_NAME.so
set -e
cd "$(dirname "$0")/../.."
V="$1"; shift
B="build_$V"
mkdir -p "$B"
FILE="${FILE:-blur_u16.hip}"
for o in build/*.o; do [ "$(basename "$o")" = "$FILE.o" ] || cp "$o" "$B/"; done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 "$@" -x hip -c "milwrm_amd/csrc/$FILE" -o "$B/$FILE.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "milwrm_amd/lib_$V.so" "$B"/*.o
echo "built milwrm_amd/lib_$V.so"
