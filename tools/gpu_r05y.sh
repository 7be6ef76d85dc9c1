#!/bin/bash
# Round 5: frame tiles (one pixel x 64 one-frame chunks per wave) for the Cornell box, 1 GPU and the
# 8-way split's every rank (emulated), vs the default 8x8 / 32x2 pixel tiles.
set -u
mkdir -p gpurun_out
: > gpurun_out/ftiles.jsonl
for env in "RT2_FRAME_TILES=0" "RT2_FRAME_TILES=1"; do
  for args in "" "--emulate-world 8 --emulate-rank all"; do
    env $env timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --stats-frames 1 $args > gpurun_out/ft_one.log 2>&1 || { tail -5 gpurun_out/ft_one.log; exit 1; }
    line=$(grep '^{' gpurun_out/ft_one.log); echo "{\"env\": \"$env\", \"args\": \"$args\", \"bench\": $line}" >> gpurun_out/ftiles.jsonl
    echo "$env [$args] $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
