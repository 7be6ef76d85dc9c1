#!/bin/bash
# Round 3: tail compaction validation + measurement (parity tests, 1-GPU / 8-way-rank benches with
# RT2_TAIL_MIN 0 vs default, launch-tail probe on the ENDTIME diagnostic build).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYK:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
: > gpurun_out/r3b.jsonl
for spec in "RT2_TAIL_MIN=0|" "RT2_TAIL_MIN=16|" "RT2_TAIL_MIN=0|--emulate-world 8 --emulate-rank 0" "RT2_TAIL_MIN=16|--emulate-world 8 --emulate-rank 0" "RT2_TAIL_MIN=32|--emulate-world 8 --emulate-rank 0" ; do
  envs="${spec%%|*}"; args="${spec#*|}"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu --steps ${STEPS:-4} --warmup 1 $args > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  line=$(grep '^{' gpurun_out/b.log)
  echo "{\"env\": \"$envs\", \"args\": \"$args\", \"bench\": $line}" >> gpurun_out/r3b.jsonl
  echo "[$envs|$args] $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
RT2_LIB=raytrace2_amd/lib/ablate/endtime.so timeout -k 10 300 python -u tools/tail_probe.py tail > gpurun_out/tail_probe.jsonl 2>gpurun_out/tail_probe.err || { tail -5 gpurun_out/tail_probe.err; exit 1; }
cat gpurun_out/tail_probe.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['world'], d['tail_min'], 'kernel_ms', d['kernel_ms'], 'span', d['span_ms'], 'tail', d['tail_ms'], 'migrated', d['migrated'])"
