#!/bin/bash
# Every BASELINE.json config on one GPU at its full size (plus one rank of an 8-way split for the
# 8-GPU configs), one bench JSON line each into gpurun_out/configs.jsonl. Stops at the first failure.
set -u
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {  # label, args...
  local label=$1; shift
  timeout -k 10 400 python bench.py --no-cpu --steps 1 --warmup 1 --stats-frames 2 "$@" > gpurun_out/cfg.log 2>&1
  local rc=$?
  local line=$(grep '^{' gpurun_out/cfg.log)
  echo "{\"config\": \"$label\", \"args\": \"$*\", \"rc\": $rc, \"bench\": ${line:-null}}" >> gpurun_out/configs.jsonl
  echo "[$label] rc=$rc $(echo "$line" | cut -c1-120)"
  case $rc in 0) ;; *) tail -5 gpurun_out/cfg.log; exit $rc;; esac
}
run "C2 cornell 1024^2 @ 1000" --steps 3
run "C3 book1 1920x1080 @ 500" --scene final_render_book_1.json --width 1920 --height 1080 --spp 500
run "C4 cornell volume 1024^2 @ 4000" --scene cornell_box_volume.json --spp 4000
run "C4 rank 0 of 8" --scene cornell_box_volume.json --spp 4000 --emulate-world 8
run "C5 book2 800^2 @ 10000" --scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000 --warmup 0
run "C5 rank 0 of 8" --scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000 --warmup 0 --emulate-world 8
run "C2 rank 0 of 8" --emulate-world 8 --steps 5
