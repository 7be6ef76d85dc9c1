#!/bin/bash
# Round 5: hit quads' transform tracked by the trace (no load of it at the trace's end: xft), then
# kernels for scenes without moving spheres take center = c0 (mot, kFeatMotion), vs commit 7c56667.
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/mot.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="qloop xft mot" REPS=2 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B2;|$B1" AB_NAME=ab_r05p bash tools/gpu_ab.sh
grep -o '"variant": [0-9]*' gpurun_out/ab_one.log
