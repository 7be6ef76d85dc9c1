#!/bin/bash
# Round 5: cost probes (each section run twice, RT2_EXP_TWICE bits) of the Cornell (v0) and book 2 (v3)
# kernels, then the wave-step diagnostic of the frame-tile scenes at representative frame counts.
set -u
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-/root/repo}
VARIANTS="v0p0 v0p1 v0p2 v0p4 v0p8 v0p16 v0p256 v0p2048" bash $R/tools/valu_probe.sh > $R/gpurun_out/probe_c2.log 2>&1 || { tail -5 $R/gpurun_out/probe_c2.log; exit 1; }
cp -r $R/gpurun_out/probe $R/gpurun_out/probe_c2_dir
cat $R/gpurun_out/probe_c2.log
VARIANTS="v3p0 v3p1 v3p2 v3p4 v3p8 v3p16 v3p32 v3p256 v3p2048" BENCH_ARGS="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000" bash $R/tools/valu_probe.sh > $R/gpurun_out/probe_c5.log 2>&1 || { tail -5 $R/gpurun_out/probe_c5.log; exit 1; }
cat $R/gpurun_out/probe_c5.log
cd $R
: > gpurun_out/wavesteps2.jsonl
for args in "scenes/book2_final_scene_10000_samples.json 128 800x800 1000" "scenes/final_render_book_1.json 128 1920x1080 500"; do
  RT2_LIB=raytrace2_amd/lib/ablate/wavesteps.so timeout -k 10 300 python tools/wavesteps.py $args > gpurun_out/ws_one.log 2>&1 || { echo "wavesteps failed: $args"; tail -5 gpurun_out/ws_one.log; exit 1; }
  cat gpurun_out/ws_one.log >> gpurun_out/wavesteps2.jsonl
done
echo done
