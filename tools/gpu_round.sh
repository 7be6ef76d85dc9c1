#!/bin/bash
# One GPU-box session: parity tests, then a short bench. Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
