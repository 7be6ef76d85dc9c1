#!/bin/bash
# rocprofv3 passes on the GPU box for the default bench workload: a kernel trace of the exact bench
# command, then one PMC pass per counter group (no tracing domains combined with --pmc).
# Outputs under gpurun_out/prof/; tools/roofline_report.py turns them into profiles/<tag>_*.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof
rm -rf $OUT; mkdir -p $OUT
PMCARGS="--no-cpu --steps 1 --warmup 0 ${BENCH_ARGS:-}"
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-200
  case $rc in 124|134|137|139) echo "crash/timeout in $name: stopping"; exit $rc;; esac
  return 0
}
run trace 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py ${BENCH_ARGS:-}
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" ; do
  name=pmc_$(echo $grp | tr ' ' '_' | cut -c1-40)
  run $name 400 rocprofv3 --pmc $grp -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py $PMCARGS
done
exit 0
