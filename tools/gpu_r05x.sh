#!/bin/bash
# Round 5: row-band height of the multi-GPU split, 8-way every rank emulated (job rate = all ranks'
# rays / slowest rank's time), C2 and C5.
set -u
mkdir -p gpurun_out
: > gpurun_out/bands.jsonl
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000"
for h in 2 4 8 16; do
  timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --stats-frames 1 --emulate-world 8 --emulate-rank all --band-h $h > gpurun_out/band_one.log 2>&1 || { tail -5 gpurun_out/band_one.log; exit 1; }
  line=$(grep '^{' gpurun_out/band_one.log); echo "{\"cfg\": \"C2 8-way h=$h\", \"bench\": $line}" >> gpurun_out/bands.jsonl
  echo "C2 h=$h $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
for h in 2 8; do
  timeout -k 10 400 python bench.py --no-cpu --steps 1 --warmup 0 --stats-frames 1 --emulate-world 8 --emulate-rank all --band-h $h $B2 > gpurun_out/band_one.log 2>&1 || { tail -5 gpurun_out/band_one.log; exit 1; }
  line=$(grep '^{' gpurun_out/band_one.log); echo "{\"cfg\": \"C5 8-way h=$h\", \"bench\": $line}" >> gpurun_out/bands.jsonl
  echo "C5 h=$h $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
