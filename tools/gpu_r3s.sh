#!/bin/bash
# One-pass box-boundary queries (Cornell volume): parity suite, then A/B base vs nopair on C4, both orders.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
C4="--scene cornell_box_volume.json --spp 1000"
AB_NAME=ab1 REPS=1 STEPS=2 VARIANTS="base nopair" CONFIGS="|$C4" bash tools/gpu_ab.sh || exit 1
AB_NAME=ab2 REPS=1 STEPS=2 VARIANTS="nopair base" CONFIGS="|$C4" bash tools/gpu_ab.sh
