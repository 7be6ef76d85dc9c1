#!/bin/bash
# Round 5: BVH-step runs branch on the wave's all-finite flag outside the lanes' exec-mask branch (fin2)
# vs commit 6e02bfc (c1first).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/fin2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="c1first fin2" REPS=2 CONFIGS="|;|$B1;|$B2" AB_NAME=ab_r05s bash tools/gpu_ab.sh
