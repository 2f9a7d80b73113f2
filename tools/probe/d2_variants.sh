#!/bin/bash
# build dense2 timing variants (CPU side): tools/probe/libd2_<name>.so.  The
# variants (wrong results: 1 = no closes, 2 = no key updates, 3 = no queue
# flushes, 4 = chunk loads + B operands only, 5 = chunk loads only) are not in
# the product kernel: d2_variants.patch adds the MW_D2_VARIANT branches to a
# copy of the sources, built with -DMW_D2_VARIANT=N.
set -e
cd "$(dirname "$0")/../.."
ROOT=$PWD
VARS=${VARS:-"noclose:-DMW_D2_VARIANT=1 noflush:-DMW_D2_VARIANT=3 bonly:-DMW_D2_VARIANT=4 lonly:-DMW_D2_VARIANT=5"}
for v in $VARS; do
  name=${v%%:*}; fl=${v#*:}
  tmp=$(mktemp -d)
  cp -rp milwrm_amd include "$tmp/"
  (cd "$tmp" && patch -s -p1 < "$ROOT/tools/probe/d2_variants.patch")
  MW_BUILD_DIR="$tmp/build" MW_LIB="$ROOT/tools/probe/libd2_$name.so" MW_EXTRA_FLAGS="$fl" \
    python -c "import sys; sys.path.insert(0, '$tmp'); from milwrm_amd.build import build; build()" > /dev/null
  rm -rf "$tmp"
  echo "built $name"
done
