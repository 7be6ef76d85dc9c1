#!/bin/bash
# Dynamic instruction counts per ray of prebuilt library variants (raytrace2_amd/lib/ablate/<v>.so):
# one rocprofv3 --pmc pass each over a short bench run; prints wave-level VALU/SALU/SMEM
# instructions per 64 rays (one wave-bounce) of the timed render dispatch.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/probe
rm -rf $OUT; mkdir -p $OUT
for v in ${VARIANTS:-base}; do
  RT2_LIB=$R/raytrace2_amd/lib/ablate/$v.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES \
    -d $OUT/$v -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --stats-frames 1 ${BENCH_ARGS:-} > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/$v.log; exit $rc;; esac
  python3 - "$OUT/$v" "$OUT/$v.log" <<'PY'
import csv, json, sys
from collections import defaultdict
d, log = sys.argv[1], sys.argv[2]
line = [l for l in open(log) if l.startswith("{")][-1]
b = json.loads(line)
rays = b["detail"]["rays"] / b["steps"]
agg = defaultdict(lambda: defaultdict(float)); dur = {}; name = {}
for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
    if "render_kernel" in r["Kernel_Name"] and ", false>" in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name[r["Dispatch_Id"]] = r["Kernel_Name"]
k = max(dur, key=lambda x: dur[x]); a = agg[k]
print(json.dumps({"Mray/s": b["value"], "ms": round(dur[k], 2), "valu_per_64rays": round(a["SQ_INSTS_VALU"] * 64 / rays, 1),
                  "salu_per_64rays": round(a["SQ_INSTS_SALU"] * 64 / rays, 1), "smem_per_64rays": round(a["SQ_INSTS_SMEM"] * 64 / rays, 1),
                  "waves": a["SQ_WAVES"], "kernel": name[k][:60]}))
PY
done
