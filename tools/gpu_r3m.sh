#!/bin/bash
# General lane walk (BVH / sphere / list-tree steps): parity suite, then A/B base vs nowalk on book 1 and book 2.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=ab1 REPS=1 STEPS=2 VARIANTS="base nowalk" CONFIGS="|$B1;|$B2" bash tools/gpu_ab.sh || exit 1
AB_NAME=ab2 REPS=1 STEPS=2 VARIANTS="nowalk base" CONFIGS="|$B1;|$B2;|--scene gen:sphere_field:20000:3 --width 1280 --height 720 --spp 64" bash tools/gpu_ab.sh
