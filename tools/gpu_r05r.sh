#!/bin/bash
# Round 5: quad-run acceptance as min(kmax, key | rejection sign) (accmin), + the transform loop of resolve_hit loading the parent link with M (c1first), vs commit 948d117 (head).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/c1first.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="head accmin c1first" REPS=2 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B2" AB_NAME=ab_r05r bash tools/gpu_ab.sh
