#!/bin/bash
# Round 5: book 2 cost probes of commit 6e02bfc (sections run twice; trtw = every ray traced twice).
set -u
mkdir -p gpurun_out
BENCH_ARGS="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000" VARIANTS="${PROBE_VARIANTS:-tw0 trtw tw8 tw16 tw32 tw1 tw2048}" bash tools/valu_probe.sh > gpurun_out/probes_r05t.log 2>&1
rc=$?
cat gpurun_out/probes_r05t.log
exit $rc
