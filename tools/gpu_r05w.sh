#!/bin/bash
# Round 5: kernel timeline of the 8-way split's rank 0 (emulated) over 8 steps, to see launch overlap.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
rm -rf $R/gpurun_out/tl_r8
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl_r8 -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 8 --warmup 2 --emulate-world 8 --emulate-rank 0 > $R/gpurun_out/tl_r8.log 2>&1
rc=$?
tail -c 300 $R/gpurun_out/tl_r8.log
exit $rc
