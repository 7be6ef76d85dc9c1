#!/bin/bash
# Final check after the SAH default (host-side tree build only; kernel unchanged): parity suite, smoke,
# C5 profile, every config's bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
TRACE_TIMEOUT=400 PMC_TIMEOUT=200 bash tools/profile.sh c5 --scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000 --steps 1 --warmup 0 || exit 1
bash tools/gpu_r3_final2.sh
