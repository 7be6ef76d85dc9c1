#!/bin/bash
# SAH-built list trees (host only, RT2_ACC_SAH=1): book-2 parity tests with it, then A/B on book 2.
set -u
mkdir -p gpurun_out
RT2_ACC_SAH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "book2 or list or c5" > gpurun_out/pytest_sah.log 2>&1; rc=$?
echo "pytest sah rc=$rc"; tail -2 gpurun_out/pytest_sah.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_sah.log | head -20; exit $rc; fi
mkdir -p raytrace2_amd/lib/ablate && cp raytrace2_amd/lib/librt2.so raytrace2_amd/lib/ablate/base.so
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
AB_NAME=ab1 REPS=2 STEPS=2 VARIANTS="base" CONFIGS="RT2_ACC_SAH=1|$B2;RT2_ACC_SAH=0|$B2" bash tools/gpu_ab.sh
