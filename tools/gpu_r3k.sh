#!/bin/bash
# Tail merge: parity suite (merge on), ENDTIME tail probes with / without merge, then A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for v in et et_nomerge; do
  echo "probe $v"
  RT2_LIB=raytrace2_amd/lib/ablate/$v.so timeout -k 10 300 python -u tools/tail_probe.py ranks > gpurun_out/tail_$v.jsonl 2>gpurun_out/tail_$v.err || { tail -5 gpurun_out/tail_$v.err; exit 1; }
  cut -c1-400 gpurun_out/tail_$v.jsonl
done
REPS=${REPS:-1} STEPS=${STEPS:-2} VARIANTS="${VARIANTS:-prev norect nomerge base}" CONFIGS="${CONFIGS:-|;|--emulate-world 8 --emulate-rank 0 --steps 6;|--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 1000}" bash tools/gpu_ab.sh
