#!/bin/bash
# Round 5: merged quad runs (book 2 kernel): parity suite with the merge on, then base vs merge (off / on).
set -u
mkdir -p gpurun_out
RT2_LIB=raytrace2_amd/lib/ablate/merge.so RT2_MERGE_RUNS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
VARIANTS="base merge" REPS=2 CONFIGS="RT2_MERGE_RUNS=0|$B2;RT2_MERGE_RUNS=1|$B2" AB_NAME=ab_r05e bash tools/gpu_ab.sh || exit 1
