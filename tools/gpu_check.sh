#!/bin/bash
# GPU-box session: the -m gpu tests (optionally a subset: TESTS="tests/x.py ..."), then bench lines
# for each argument string ("" = default). Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
fi
LINES=gpurun_out/${LINES_NAME:-bench_lines}.jsonl
: > $LINES
for args in "$@"; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  line=$(grep '^{' gpurun_out/bench_one.log)
  echo "{\"args\": \"$args\", \"rc\": $rc, \"bench\": ${line:-null}}" >> $LINES
  echo "bench [$args] rc=$rc $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['detail']['gather_ms_per_step'], (d['roofline'] or {}).get('avg_launch_ms'), (d['cpu_baseline'] or {}).get('value'))" 2>/dev/null)"
  case $rc in 0) ;; *) tail -8 gpurun_out/bench_one.log; exit $rc;; esac
done
