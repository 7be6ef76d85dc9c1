#!/bin/bash
# Bench sweep with per-line environment: each argument is "VAR=v VAR2=w ... -- bench args".
# Lines go to gpurun_out/${LINES_NAME:-sweep}.jsonl. Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
LINES=gpurun_out/${LINES_NAME:-sweep}.jsonl
: > $LINES
for spec in "$@"; do
  envs="${spec%%--*}"; args="${spec#*--}"
  env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py --no-cpu $args > gpurun_out/sweep_one.log 2>&1
  rc=$?
  line=$(grep '^{' gpurun_out/sweep_one.log)
  echo "{\"env\": \"$envs\", \"args\": \"$args\", \"rc\": $rc, \"bench\": ${line:-null}}" >> $LINES
  echo "[$envs|$args] rc=$rc $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['work_split'], [r['ms_per_step'] for r in d['detail']['per_rank']])" 2>/dev/null)"
  case $rc in 0) ;; *) tail -8 gpurun_out/sweep_one.log; exit $rc;; esac
done
