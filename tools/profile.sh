#!/bin/bash
# rocprofv3 passes on the GPU box: kernel trace of the default bench, then PMC passes (one
# counter group per pass, no tracing domains combined with --pmc). Outputs under gpurun_out/prof/.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
SHORT="--spp 64 --steps 1 --warmup 0 --no-cpu --stats-frames 4"
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  case $rc in 124|134|137|139) echo "crash/timeout in $name: stopping"; exit $rc;; esac
  return 0
}
run trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py ${BENCH_ARGS:-}
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM" ; do
  name=pmc_$(echo $grp | tr ' ' '_' | cut -c1-40)
  run $name 300 rocprofv3 --pmc $grp -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py $SHORT
done
exit 0
