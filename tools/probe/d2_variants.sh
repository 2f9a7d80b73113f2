#!/bin/bash
# build dense2 timing variants (CPU side): libd2_<name>.so with -D flags
set -e
cd "$(dirname "$0")/../.."
for v in "base:" "noclose:-DMW_D2_VARIANT=1" "nokeys:-DMW_D2_VARIANT=2" "noflush:-DMW_D2_VARIANT=3"; do
  name=${v%%:*}; fl=${v#*:}
  rm -rf "build_d2_$name"; cp -rp build "build_d2_$name"; rm -f "build_d2_$name/lloyd.hip.o"
  MW_BUILD_DIR="build_d2_$name" MW_LIB="tools/probe/libd2_$name.so" MW_EXTRA_FLAGS="$fl" python -c "from milwrm_amd.build import build; build()" > /dev/null
  echo "built $name"
done
