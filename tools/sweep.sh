#!/bin/bash
# Parity tests, then one bench line per argument set ("--no-cpu" added), e.g.
#   tools/sweep.sh "--work-split 0" "--work-split 8" "--emulate-world 8 --work-split 8"
# Stops at the first crash/timeout. Lines go to gpurun_out/sweep.jsonl.
set -u
mkdir -p gpurun_out
: > gpurun_out/sweep.jsonl
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for args in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-2} --warmup 1 $args > gpurun_out/sweep_one.log 2>&1
  rc=$?
  line=$(grep '^{' gpurun_out/sweep_one.log)
  echo "{\"args\": \"$args\", \"rc\": $rc, \"bench\": ${line:-null}}" >> gpurun_out/sweep.jsonl
  echo "[$args] rc=$rc"; echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['work_split'], d['detail']['launches'])" 2>/dev/null || tail -5 gpurun_out/sweep_one.log
  case $rc in 0) ;; *) exit $rc;; esac
done
