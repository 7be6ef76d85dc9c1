#!/bin/bash
# Octant-ordered list-tree copies: parity suite (on), then A/B RT2_ACC_OCTANTS=1 vs 0 on book 2, both orders.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
mkdir -p raytrace2_amd/lib/ablate && cp raytrace2_amd/lib/librt2.so raytrace2_amd/lib/ablate/base.so
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=ab1 REPS=2 STEPS=2 VARIANTS="base" CONFIGS="RT2_ACC_OCTANTS=1|$B2;RT2_ACC_OCTANTS=0|$B2" bash tools/gpu_ab.sh
