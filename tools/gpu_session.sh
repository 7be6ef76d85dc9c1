#!/bin/bash
# One GPU-box session (the single launcher for gpurun; it replaces round 5's per-experiment scripts,
# whose results are in profiles/). Steps run in the order given and the session stops at the first
# failure, so nothing more touches the GPU after a fault, abort or time limit:
#   tools/gpu_session.sh tests [bench] [bench20] [configs] [profile] [ab] [lines]
#     tests     -m gpu suite (TESTS="tests/x.py ..." for a subset; PYTEST_TIMEOUT for the whole step)
#     bench     bench.py --steps 3 (BENCH_ARGS appended)
#     bench20   the driver's command: bench.py --gpus 1 --steps 20 --warmup 5 (BENCH_ARGS appended)
#     configs   every BASELINE config + emulated splits (tools/bench_configs.sh -> configs.jsonl)
#     profile   rocprofv3 trace + PMC passes of every config (tools/profile_all.sh)
#     ab        A/B of prebuilt variants (VARIANTS, CONFIGS, REPS, AB_NAME: tools/gpu_ab.sh)
#     lines     one bench line per element of LINES_ARGS (';'-separated) -> gpurun_out/lines.jsonl
# Output goes to gpurun_out/ (merged back by gpurun).
set -u
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
stop() { echo "stopping after $1 (rc=$2)"; exit $2; }
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider \
        --timeout ${TEST_TIMEOUT:-300} --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      rc=$?
      echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
      if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; stop tests $rc; fi ;;
    bench|bench20)
      if [ $step = bench ]; then a="--steps 3 --warmup 1"; else a="--gpus 1 --steps 20 --warmup 5"; fi
      timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $a ${BENCH_ARGS:-} > gpurun_out/$step.log 2>&1
      rc=$?
      echo "$step rc=$rc"; grep '^{' gpurun_out/$step.log | cut -c1-1500
      [ $rc -eq 0 ] || { tail -8 gpurun_out/$step.log; stop $step $rc; } ;;
    configs)
      bash $R/tools/bench_configs.sh || stop configs $? ;;
    profile)
      bash $R/tools/profile_all.sh > gpurun_out/profile_all.log 2>&1
      rc=$?
      cut -c1-200 gpurun_out/profile_all.log
      [ $rc -eq 0 ] || stop profile $rc ;;
    ab)
      bash $R/tools/gpu_ab.sh || stop ab $? ;;
    lines)
      : > gpurun_out/lines.jsonl
      IFS=';' read -ra LA <<< "${LINES_ARGS:-}"
      for args in "${LA[@]}"; do
        timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $args > gpurun_out/line_one.log 2>&1
        rc=$?
        line=$(grep '^{' gpurun_out/line_one.log)
        echo "{\"args\": \"$args\", \"rc\": $rc, \"bench\": ${line:-null}}" >> gpurun_out/lines.jsonl
        echo "[$args] rc=$rc $(echo "$line" | cut -c1-300)"
        [ $rc -eq 0 ] || { tail -8 gpurun_out/line_one.log; stop lines $rc; }
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
