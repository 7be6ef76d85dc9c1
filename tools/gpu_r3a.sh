#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/b1.log 2>&1 || exit $?
grep '^{' gpurun_out/b1.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-cpu --steps 1 --warmup 1 --scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 2000 > gpurun_out/b2.log 2>&1 || exit $?
grep '^{' gpurun_out/b2.log | cut -c1-400
