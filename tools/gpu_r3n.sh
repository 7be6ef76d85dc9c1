#!/bin/bash
# Pruned list-walk kernel: parity suite, then book 2 A/B: head vs pruned (base) vs 7 waves, frame tiles on/off.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=ab1 REPS=1 STEPS=2 VARIANTS="head base w7" CONFIGS="|$B2;RT2_FRAME_TILES=0|$B2" bash tools/gpu_ab.sh || exit 1
AB_NAME=ab2 REPS=1 STEPS=2 VARIANTS="w7 base head" CONFIGS="|$B2;RT2_FRAME_TILES=0|$B2" bash tools/gpu_ab.sh
