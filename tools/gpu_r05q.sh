#!/bin/bash
# Round 5: kFeatMotion alone (mot2) vs commit 7c56667 (qloop).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/mot2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="qloop mot2" REPS=2 CONFIGS="|;|$B2;|$B1" AB_NAME=ab_r05q bash tools/gpu_ab.sh
