#!/bin/bash
# Dev variant of the library with only blur_u16.hip rebuilt (radius 8 only,
# -DMW_BLUR_DEV) under extra flags; every other object is reused from build/.
#   bash tools/dev/build_variant.sh NAME [-DFLAG ...]  ->  milwrm_amd/lib_NAME.so
set -e
cd "$(dirname "$0")/../.."
V="$1"; shift
B="build_$V"
mkdir -p "$B"
for o in build/*.o; do [ "$(basename "$o")" = blur_u16.hip.o ] || cp "$o" "$B/"; done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -DMW_BLUR_DEV "$@" -x hip -c milwrm_amd/csrc/blur_u16.hip -o "$B/blur_u16.hip.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "milwrm_amd/lib_$V.so" "$B"/*.o
echo "built milwrm_amd/lib_$V.so"
