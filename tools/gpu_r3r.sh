#!/bin/bash
# Host-side knob sweep on the final kernel: frame-tile chunk length and BVH pairing (book 2, book 1).
set -u
mkdir -p gpurun_out raytrace2_amd/lib/ablate
cp raytrace2_amd/lib/librt2.so raytrace2_amd/lib/ablate/base.so
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=sweep REPS=2 STEPS=2 VARIANTS="base" CONFIGS="|$B2;RT2_FRAME_TILE_LEN=4|$B2;RT2_FRAME_TILE_LEN=16|$B2;RT2_BVH_PAIRS=0|$B2;|$B1;RT2_FRAME_TILE_LEN=4|$B1;RT2_FRAME_TILE_LEN=16|$B1" bash tools/gpu_ab.sh
