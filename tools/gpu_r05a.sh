#!/bin/bash
# Round 5: GPU parity suite, then the driver's bench command (20 steps). Stops at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench20.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench20.log | cut -c1-3000
exit $rc
