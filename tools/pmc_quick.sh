#!/bin/bash
# PMC passes (one counter group per run) over one bench configuration: BENCH_ARGS="...".
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmcq
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-200} rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 ${BENCH_ARGS:-} > $OUT/g$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/g$i.log; exit $rc;; esac
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in glob.glob(out + "/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "render_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4e} dispatches={len(disp[k])}")
PY
