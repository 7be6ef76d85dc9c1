#!/bin/bash
# A/B of prebuilt library variants (raytrace2_amd/lib/ablate/<v>.so) on bench configurations:
#   VARIANTS="a b" CONFIGS="ENV=1|--args;..." tools/gpu_ab.sh   -> gpurun_out/ab.jsonl
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${AB_NAME:-ab}.jsonl
: > $OUT
IFS=';' read -ra CFGS <<< "${CONFIGS:-|}"
for rep in $(seq 1 ${REPS:-1}); do
for cfg in "${CFGS[@]}"; do
  envs="${cfg%%|*}"; args="${cfg#*|}"
  for v in ${VARIANTS}; do
    env $envs RT2_LIB=raytrace2_amd/lib/ablate/$v.so timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py --no-cpu --steps ${STEPS:-3} --warmup 1 --stats-frames 1 $args > gpurun_out/ab_one.log 2>&1 || { echo "FAILED $v $cfg"; tail -5 gpurun_out/ab_one.log; exit 1; }
    line=$(grep '^{' gpurun_out/ab_one.log)
    echo "{\"variant\": \"$v\", \"env\": \"$envs\", \"args\": \"$args\", \"rep\": $rep, \"bench\": $line}" >> $OUT
    echo "$v [$envs|$args] $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
  done
done
done
