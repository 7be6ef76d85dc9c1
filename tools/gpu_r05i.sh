#!/bin/bash
# Round 5 probe: every scalar step/record load issued twice (latency exposed twice) vs the kernel.
set -u
mkdir -p gpurun_out
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base sld2" REPS=2 CONFIGS="|;|$B1;|$B2" AB_NAME=ab_r05i bash tools/gpu_ab.sh
