#!/bin/bash
# Round 5: C2 cost probes of the kernel at commit 7c56667 (RT2_EXP_TWICE sections run twice).
set -u
mkdir -p gpurun_out
VARIANTS="tw0 tw1 tw2 tw4 tw8 tw16 tw256 tw512 tw2048" bash tools/valu_probe.sh > gpurun_out/probes_r05o.log 2>&1
rc=$?
cat gpurun_out/probes_r05o.log
exit $rc
