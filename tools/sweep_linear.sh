#!/bin/bash
# Threaded (lockstep) vs stack traversal on programs longer than kLinearMaxSteps: the same bench
# lines with RT2_LINEAR_MAX_STEPS raised (parity tests first, under the raised limit).
# Lines go to gpurun_out/sweep_{stack,linear}.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ -z "${NO_TESTS:-}" ]; then
  RT2_LINEAR_MAX_STEPS=${LIN:-1000000} timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_linear.log 2>&1
  rc=$?
  echo "pytest (linear limit ${LIN:-1000000}) rc=$rc"; tail -15 gpurun_out/pytest_gpu_linear.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
G="--width 1920 --height 1080 --spp 64"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000"
set -- "$B2" "--scene gen:sphere_field:100000:1 $G" "--scene gen:sphere_field:10000:1 $G" "${@}"
NO_TESTS=1 STEPS=1 bash tools/sweep.sh "$@" || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_stack.jsonl
RT2_LINEAR_MAX_STEPS=${LIN:-1000000} NO_TESTS=1 STEPS=1 bash tools/sweep.sh "$@" || exit $?
cp gpurun_out/sweep.jsonl gpurun_out/sweep_linear.jsonl
