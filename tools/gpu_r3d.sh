#!/bin/bash
# Full GPU parity suite, default bench, launch-tail probe (ENDTIME build) and the Cornell-volume
# cost probes (RT2_EXP_TWICE variants, PMC instruction counts per ray).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
grep '^{' gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['detail']['runtime'])"
RT2_LIB=raytrace2_amd/lib/ablate/endtime.so timeout -k 10 300 python -u tools/tail_probe.py ranks > gpurun_out/tail_probe.jsonl 2>gpurun_out/tail_probe.err || { tail -5 gpurun_out/tail_probe.err; exit 1; }
cat gpurun_out/tail_probe.jsonl
VARIANTS="base t1 t2 t4 t8 t16 t32 t64 t128" BENCH_ARGS="--scene cornell_box_volume.json --spp 1000" timeout -k 10 900 bash tools/valu_probe.sh > gpurun_out/valu_probe_c4.log 2>&1; rc=$?
grep -v "^\s*$" gpurun_out/valu_probe_c4.log | tail -20; exit $rc
