#!/bin/bash
# Parity tests + default bench (no CPU leg). Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for args in "${@:-}"; do
  timeout -k 10 300 python bench.py --no-cpu $args > gpurun_out/bench_quick.log 2>&1
  rc=$?
  echo "bench [$args] rc=$rc"; grep '^{' gpurun_out/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['detail'])" || tail -5 gpurun_out/bench_quick.log
  case $rc in 0) ;; *) exit $rc;; esac
done
