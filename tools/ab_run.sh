#!/bin/bash
# GPU-box A/B session: optional -m gpu tests (TESTS="..."), then sweep_env lines given as arguments.
set -u
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
fi
bash tools/sweep_env.sh "$@"
