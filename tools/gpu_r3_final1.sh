#!/bin/bash
# Round-3 final kernel: parity suite, then every config's rocprofv3 trace + PMC passes (profile_all.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
bash tools/profile_all.sh
