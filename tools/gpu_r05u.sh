#!/bin/bash
# Round 5: accelerated lists walked while-while (ww) vs commit bf98a53 (c1first).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/ww.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="c1first ww" REPS=2 CONFIGS="|$B2;|" AB_NAME=ab_r05u bash tools/gpu_ab.sh
