#!/bin/bash
# Round 5 final kernel: every BASELINE config (tools/bench_configs.sh), then the driver's bench command.
set -u
mkdir -p gpurun_out
bash tools/bench_configs.sh || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1
rc=$?
tail -1 gpurun_out/bench_default.log | cut -c1-400
exit $rc
