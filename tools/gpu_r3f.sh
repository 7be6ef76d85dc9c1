#!/bin/bash
# Selftests, volume parity with the div_by_inv box-boundary variant, then the volume A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_selftest.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_self.log 2>&1 || { tail -20 gpurun_out/pytest_self.log; exit 1; }
tail -1 gpurun_out/pytest_self.log
for v in dinv v8dinv; do
RT2_LIB=raytrace2_amd/lib/ablate/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "volume or c4" > gpurun_out/pytest_$v.log 2>&1 || { tail -20 gpurun_out/pytest_$v.log; exit 1; }
echo "$v parity: $(tail -1 gpurun_out/pytest_$v.log)"
done
STEPS=2 VARIANTS="base dinv v8 v8dinv" CONFIGS="|--scene cornell_box_volume.json --spp 1000;|--scene cornell_box_volume.json --spp 4000 --emulate-world 8 --emulate-rank 0" bash tools/gpu_ab.sh
