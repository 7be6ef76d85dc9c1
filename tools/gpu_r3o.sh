#!/bin/bash
# Experiment: full per-lane walk (walkq: with quad runs; walk2: without) vs base on book 1 / book 2; parity of walkq.
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/walkq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_walkq.log 2>&1; rc=$?
echo "pytest walkq rc=$rc"; tail -2 gpurun_out/pytest_walkq.log
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=ab1 REPS=1 STEPS=2 VARIANTS="base walkq walk2" CONFIGS="|$B2;|$B1" bash tools/gpu_ab.sh || exit 1
AB_NAME=ab2 REPS=1 STEPS=2 VARIANTS="walk2 walkq base" CONFIGS="|$B2;|$B1" bash tools/gpu_ab.sh
