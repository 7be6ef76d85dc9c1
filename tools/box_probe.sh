#!/bin/bash
# Round 6: cost of a box-level MakeBox test against the six-face quad run.
# Variants (tools/build_variants.sh): base, box (RT2_EXP_TWICE=8192: the box-level test computed beside
# every MakeBox run, result discarded), quad2 (RT2_EXP_TWICE=16: every quad-run test twice). PMC
# instruction counts (tools/valu_probe.sh) and A/B timing (tools/gpu_ab.sh) on C2 and book 2 at spp 1000.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
for cfg in "" "$B2"; do
  VARIANTS="base box quad2" BENCH_ARGS="$cfg" bash $R/tools/valu_probe.sh || exit 1
done
VARIANTS="base box quad2" REPS=2 CONFIGS="|;|$B2" AB_NAME=ab_r06_box bash $R/tools/gpu_ab.sh
