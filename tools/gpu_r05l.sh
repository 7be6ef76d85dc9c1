#!/bin/bash
# Round 5: QUADAA test as one rejection word (signor2: bounds, |d_K| and the interval key folded) vs
# the bounds' sign word only (signor) vs four compares (qrange2).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/signor2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="qrange2 signor signor2" REPS=2 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B2" AB_NAME=ab_r05l bash tools/gpu_ab.sh
