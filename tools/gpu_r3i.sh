#!/bin/bash
# Parity suite on the default build (book 2 parks its path state in LDS), then A/B park vs nopark on book 2.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
REPS=${REPS:-2} STEPS=${STEPS:-2} VARIANTS="${VARIANTS:-base nopark noaccfma}" CONFIGS="${CONFIGS:-|--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000}" bash tools/gpu_ab.sh
