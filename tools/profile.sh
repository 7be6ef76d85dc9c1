#!/bin/bash
# rocprofv3 passes on the GPU box for one bench configuration:
#   tools/profile.sh <name> [bench args...]
# a kernel trace (--kernel-trace --stats) of the bench command, then one PMC pass per counter group
# (no tracing domains combined with --pmc; each pass its own run), into gpurun_out/prof_<name>/.
# tools/roofline_report.py <tag> <name> turns them into profiles/<tag>_<name>_{kernel_stats.csv,summary.json}.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=$1; shift
OUT=$R/gpurun_out/prof_$NAME
rm -rf $OUT; mkdir -p $OUT
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$NAME] $name rc=$rc $(grep '^{' $OUT/$name.log | cut -c1-160)"
  case $rc in 0) ;; *) echo "failed in $name: stopping"; tail -5 $OUT/$name.log; exit $rc;; esac
}
run trace ${TRACE_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@"
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" ; do
  name=pmc_$(echo $grp | tr ' ' '_' | cut -c1-40)
  run $name ${PMC_TIMEOUT:-300} rocprofv3 --pmc $grp -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 "$@"
done
exit 0
