#!/bin/bash
# Round 5: quad-run loop with an end bit in the codes, a byte offset and a VGPR ref counter (qloop) vs
# the kProgramEnd build (base2 = commit 29fa10a).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/qloop.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base2 qloop" REPS=2 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B2" AB_NAME=ab_r05n bash tools/gpu_ab.sh
