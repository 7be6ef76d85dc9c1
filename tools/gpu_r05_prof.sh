#!/bin/bash
# Round 5 final kernel: GPU parity suite, then every config's rocprofv3 kernel trace + PMC passes.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/profile_all.sh > gpurun_out/profile_all.log 2>&1
rc=$?
cat gpurun_out/profile_all.log | cut -c1-200
exit $rc
