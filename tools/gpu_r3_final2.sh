#!/bin/bash
# Round-3 final kernel: one bench line per BASELINE config (bench_configs.sh), the default bench, smoke.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/bench_configs.sh
