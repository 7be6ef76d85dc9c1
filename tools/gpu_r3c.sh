#!/bin/bash
# Tail compaction: parity subset, then A/B of headk (kernel without it) vs two (current) and the
# launch-tail probe on the ENDTIME build.
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "tail or work_split" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in two_endtime; do RT2_LIB=raytrace2_amd/lib/ablate/$v.so timeout -k 10 300 python -u tools/tail_probe.py tail > gpurun_out/tail_$v.jsonl 2>gpurun_out/tail_probe.err || { tail -5 gpurun_out/tail_probe.err; exit 1; }
echo $v; python3 -c "
import json,sys
for l in open('gpurun_out/tail_$v.jsonl'):
    d=json.loads(l); print(d['world'], d['tail_min'], 'kernel_ms', d['kernel_ms'], 'span', d['span_ms'], 'tail', d['tail_ms'], 'migrated', d['migrated'], d['resumed'])"; done
VARIANTS="${VARIANTS:-headk two}" CONFIGS="${CONFIGS:-RT2_TAIL_MIN=0|;RT2_TAIL_MIN=16|;RT2_TAIL_MIN=0|--emulate-world 8 --emulate-rank 0;RT2_TAIL_MIN=16|--emulate-world 8 --emulate-rank 0}" bash tools/gpu_ab.sh || exit 1
