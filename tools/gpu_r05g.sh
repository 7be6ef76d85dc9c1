#!/bin/bash
# Round 5: A/B of the still-sphere and disc-sqrt changes separately (book 1, book 2).
set -u
mkdir -p gpurun_out
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base NO_SQFAST NO_STILL still" REPS=2 CONFIGS="|$B1;|$B2" AB_NAME=ab_r05g bash tools/gpu_ab.sh
