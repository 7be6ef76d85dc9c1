#!/bin/bash
# Round 5 probe: book 2's threaded kernel at 8 (default: LDS Philox block, parked path state, 12-B sample
# stores) / 7 / 6 / 5 waves per SIMD (no LDS Philox, no parking, octet sample staging), final kernel.
set -u
mkdir -p gpurun_out
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base b2w7 b2w6 b2w5" REPS=2 CONFIGS="|$B2" AB_NAME=ab_r05z bash tools/gpu_ab.sh
