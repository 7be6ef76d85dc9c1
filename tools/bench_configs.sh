#!/bin/bash
# Every BASELINE.json config on one GPU at its full size, plus the 8-GPU configs' 8-way row-band
# split emulated rank by rank on this GPU (job rate = all ranks' rays / the slowest rank's time, no
# gather), one bench JSON line each into gpurun_out/configs.jsonl. Stops at the first failure.
set -u
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {  # label, args...
  local label=$1; shift
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --no-cpu --steps 1 --warmup 1 --stats-frames 2 "$@" > gpurun_out/cfg.log 2>&1
  local rc=$?
  local line=$(grep '^{' gpurun_out/cfg.log)
  echo "{\"config\": \"$label\", \"args\": \"$*\", \"rc\": $rc, \"bench\": ${line:-null}}" >> gpurun_out/configs.jsonl
  echo "[$label] rc=$rc $(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('frac'), r.get('valu_issue_frac'), r.get('hbm_frac'), r.get('profile'))" 2>/dev/null)"
  case $rc in 0) ;; *) tail -5 gpurun_out/cfg.log; exit $rc;; esac
}
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 500"
VOL="--scene cornell_box_volume.json --spp 4000"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000"
run "C1 cornell 400^2 @ 64" --width 400 --height 400 --spp 64 --steps 5
run "C2 cornell 1024^2 @ 1000" --steps 3
# (a rank's step is a 20-40 ms launch: 10 steps after 2 warm-up ones, as the driver's runs do many)
run "C2 8-way, every rank" --steps 10 --warmup 2 --emulate-world 8 --emulate-rank all
run "C2 4-way, every rank" --steps 10 --warmup 2 --emulate-world 4 --emulate-rank all
run "C2 2-way, every rank" --steps 5 --warmup 2 --emulate-world 2 --emulate-rank all
run "C3 book1 1920x1080 @ 500" $B1 --steps 2
run "C4 cornell volume 1024^2 @ 4000" $VOL
run "C4 8-way, every rank" $VOL --emulate-world 8 --emulate-rank all --warmup 1
run "C5 book2 800^2 @ 10000" $B2 --warmup 0
run "C5 8-way, every rank" $B2 --emulate-world 8 --emulate-rank all --warmup 1 --steps 2
