#!/bin/bash
# build dense2 timing variants (CPU side): tools/probe/libd2_<name>.so with -D flags
# (run after a main build: only lloyd.hip is recompiled per variant)
set -e
cd "$(dirname "$0")/../.."
VARS=${VARS:-"noclose:-DMW_D2_VARIANT=1 noflush:-DMW_D2_VARIANT=3 bonly:-DMW_D2_VARIANT=4 lonly:-DMW_D2_VARIANT=5"}
for v in $VARS; do
  name=${v%%:*}; fl=${v#*:}
  rm -rf "build_d2_$name"; cp -rp build "build_d2_$name"; rm -f "build_d2_$name/lloyd.hip.o"
  MW_BUILD_DIR="build_d2_$name" MW_LIB="tools/probe/libd2_$name.so" MW_EXTRA_FLAGS="$fl" python -c "from milwrm_amd.build import build; build()" > /dev/null
  echo "built $name"
done
