#!/bin/bash
# Round 5 probe: wave priority raised (s_setprio 1 / 3) while a hit is resolved, vs commit 5849eec (base).
set -u
mkdir -p gpurun_out
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base prio1 prio3" REPS=2 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B2;|$B1" AB_NAME=ab_r05v bash tools/gpu_ab.sh
