#!/bin/bash
# Parity suite on the default build, then A/B of run blocks (base) vs none (nrb) on every config.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
STEPS=${STEPS:-2} VARIANTS="${VARIANTS:-base nrb}" CONFIGS="${CONFIGS:-|;|--scene cornell_box_volume.json --spp 1000;|--scene final_render_book_1.json --width 1920 --height 1080 --spp 100;|--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000}" bash tools/gpu_ab.sh
