#!/bin/bash
# Register / spill table of one threaded product kernel (fast compile of that instantiation only):
#   tools/regs.sh <variant index 0..4> [extra hipcc flags...]
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
V=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -mllvm -structurizecfg-skip-uniform-regions=true -mllvm -simplifycfg-sink-common=false -DRT2_ONLY_VARIANT=$V "$@" \
  -S --cuda-device-only -o /tmp/rt2_regs_$V.s $R/raytrace2_amd/csrc/render.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
  | python3 $R/tools/resources.py | grep -E "mode=2 stats=0"
