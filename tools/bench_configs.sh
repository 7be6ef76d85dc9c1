set -u
mkdir -p gpurun_out
for args in "--scene final_render_book_1.json --width 1920 --height 1080 --spp 500 --launch-frames 50" "--scene cornell_box_volume.json --spp 4000 --launch-frames 200" "--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000 --launch-frames 100"; do
  timeout -k 10 240 python bench.py --no-cpu --steps 1 --warmup 0 $args > gpurun_out/cfg.log 2>&1
  rc=$?
  echo "[$args] rc=$rc"
  grep '^{' gpurun_out/cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['records_per_ray'], d['detail']['rays_per_sample'])" || tail -3 gpurun_out/cfg.log
  case $rc in 0) ;; *) exit $rc;; esac
done
