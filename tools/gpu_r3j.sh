#!/bin/bash
# Parity suite on the default build (rectangle quad codes), then A/B rect vs norect on C2, C4, C5.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
REPS=${REPS:-2} STEPS=${STEPS:-2} VARIANTS="${VARIANTS:-base norect}" CONFIGS="${CONFIGS:-|;|--scene cornell_box_volume.json --spp 1000;|--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000}" bash tools/gpu_ab.sh
