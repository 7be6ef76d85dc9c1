#!/bin/bash
# Round 5: parity suite (current build: the lane walk at RT2_LANE_SUBTREE=32), A/B of builds on every
# config, the lane-subtree sweep on book 1 / book 2, wave-step diagnostics.
set -u
mkdir -p gpurun_out
RT2_LANE_SUBTREE=32 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 100"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="key allaa sel" REPS=1 CONFIGS="|;|--scene cornell_box_volume.json --spp 1000;|$B1;|$B2" AB_NAME=ab_r05c bash tools/gpu_ab.sh || exit 1
VARIANTS="sel" REPS=1 CONFIGS="RT2_LANE_SUBTREE=8|$B2;RT2_LANE_SUBTREE=16|$B2;RT2_LANE_SUBTREE=32|$B2;RT2_LANE_SUBTREE=64|$B2;RT2_LANE_SUBTREE=128|$B2;RT2_LANE_SUBTREE=16|$B1;RT2_LANE_SUBTREE=64|$B1" AB_NAME=ab_r05c_lane bash tools/gpu_ab.sh || exit 1
: > gpurun_out/wavesteps.jsonl
for args in "scenes/book2_final_scene_10000_samples.json 8 800x800 1000" "scenes/cornell_box_original.json 16 1024x1024 1000" "scenes/final_render_book_1.json 4 1920x1080 500"; do
  RT2_LIB=raytrace2_amd/lib/ablate/wavesteps.so timeout -k 10 300 python tools/wavesteps.py $args > gpurun_out/ws_one.log 2>&1 || { echo "wavesteps failed: $args"; tail -5 gpurun_out/ws_one.log; exit 1; }
  cat gpurun_out/ws_one.log >> gpurun_out/wavesteps.jsonl
  cat gpurun_out/ws_one.log
done
