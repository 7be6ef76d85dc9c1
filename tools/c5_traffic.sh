#!/bin/bash
# Book 2 (C5) HBM traffic attribution: FETCH_SIZE / WRITE_SIZE passes of one render step (spp 1000)
# with the accelerated list's tree in one copy (RT2_ACC_OCTANTS=0) and in eight octant copies; RT2_LIB
# (absolute path) selects a build, e.g. the RT2_EXP_NOSTORE=1 diagnostic; TAG names the output dir.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-c5traffic}
rm -rf $OUT; mkdir -p $OUT
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp ${SPP:-1000}"
for oct in ${OCTS:-1 0}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RT2_ACC_OCTANTS=$oct RT2_LIB=${RT2_LIB:-$R/raytrace2_amd/lib/librt2.so} timeout -k 10 240 rocprofv3 --pmc $c -d $OUT/o${oct}_$c -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --stats-frames 1 $B2 > $OUT/o${oct}_$c.log 2>&1
    rc=$?; echo "oct=$oct $c rc=$rc"
    case $rc in 0) ;; *) tail -5 $OUT/o${oct}_$c.log; exit $rc;; esac
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, os
out = sys.argv[1]
for d in sorted(glob.glob(out + "/o*_*")):
    if not os.path.isdir(d): continue
    log = d + ".log"
    line = [l for l in open(log) if l.startswith("{")][-1]
    b = json.loads(line); rays = b["detail"]["rays"]
    tot = 0.0
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_kernel" in r["Kernel_Name"] and ", false>" in r["Kernel_Name"]:
                tot += float(r["Counter_Value"])
    print(os.path.basename(d), f"{tot:.4e}", "per ray", round(tot * 1024 / rays, 2) if "SIZE" in d else None, "rays", rays)
PY
