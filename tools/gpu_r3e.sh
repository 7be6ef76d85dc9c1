#!/bin/bash
# Full parity suite, then bench lines for C2 / C4 / C5 (short) and the volume PMC instruction counts.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for args in "" "--scene cornell_box_volume.json --spp 1000" "--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 2000 --steps 1"; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 $args > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  grep '^{' gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['config']['workload'], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
VARIANTS="base" BENCH_ARGS="--scene cornell_box_volume.json --spp 1000" timeout -k 10 300 bash tools/valu_probe.sh > gpurun_out/valu_probe_c4b.log 2>&1; rc=$?
grep -v "^\s*$" gpurun_out/valu_probe_c4b.log | tail -3; exit $rc
