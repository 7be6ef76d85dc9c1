#!/bin/bash
# Round 5: parity suite with merged sphere steps, A/B against the committed kernel, wave steps of book 1.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base msph" REPS=2 CONFIGS="|$B1;|$B2;|" AB_NAME=ab_r05h bash tools/gpu_ab.sh || exit 1
RT2_LIB=raytrace2_amd/lib/ablate/ws_msph.so timeout -k 10 300 python tools/wavesteps.py scenes/final_render_book_1.json 128 1920x1080 500 > gpurun_out/ws_msph.log 2>&1; echo "ws rc=$?"; tail -30 gpurun_out/ws_msph.log
