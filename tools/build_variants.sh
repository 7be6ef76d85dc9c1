#!/bin/bash
# Builds librt2.so variants (name:flag,flag ...) into raytrace2_amd/lib/ablate/<name>.so, then
# rebuilds the default library. Usage: tools/build_variants.sh "c8:-DRT2_MIN_WAVES_CORNELL=8" ...
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/raytrace2_amd/lib/ablate
for v in "$@"; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr "," " ")
  make -s -C $R/raytrace2_amd/csrc clean >/dev/null
  make -s -j8 -C $R/raytrace2_amd/csrc HIPFLAGS_EXTRA="$flags" >/dev/null 2>&1 || { echo "build $name failed"; exit 1; }
  cp $R/raytrace2_amd/lib/librt2.so $R/raytrace2_amd/lib/ablate/$name.so
done
make -s -C $R/raytrace2_amd/csrc clean >/dev/null; make -s -j8 -C $R/raytrace2_amd/csrc >/dev/null 2>&1 || exit 1
cp $R/raytrace2_amd/lib/librt2.so $R/raytrace2_amd/lib/ablate/base.so
ls $R/raytrace2_amd/lib/ablate
