#!/bin/bash
# Build (here) ablation variants of librt2.so into build/ablate/<name>.so; run (GPU box) each with bench.
set -u
MODE=${1:-run}
R=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS="${VARIANTS_LIST:-base: noballot:-DRT2_EXP_NO_BALLOT=1 cheaprng:-DRT2_EXP_CHEAP_RNG=1 fastdiv:-DRT2_EXP_FAST_DIV=1} ${EXTRA_VARIANTS:-}"
if [ "$MODE" = build ]; then
  mkdir -p $R/raytrace2_amd/lib/ablate
  for v in $VARIANTS; do
    name=${v%%:*}; flags=$(echo "${v#*:}" | tr "," " ")
    make -s -C $R/raytrace2_amd/csrc clean >/dev/null
    make -s -j8 -C $R/raytrace2_amd/csrc HIPFLAGS_EXTRA="$flags" >/dev/null || exit 1
    cp $R/raytrace2_amd/lib/librt2.so $R/raytrace2_amd/lib/ablate/$name.so
  done
  make -s -C $R/raytrace2_amd/csrc clean >/dev/null; make -s -j8 -C $R/raytrace2_amd/csrc >/dev/null
  ls $R/raytrace2_amd/lib/ablate; exit 0
fi
mkdir -p $R/gpurun_out
for v in $VARIANTS; do
  name=${v%%:*}
  RT2_LIB=$R/raytrace2_amd/lib/ablate/$name.so timeout -k 10 200 python $R/bench.py --no-cpu --steps 2 --warmup 1 ${BENCH_ARGS:-} > $R/gpurun_out/ablate_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep '^{' $R/gpurun_out/ablate_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mray/s", d["roofline"]["avg_launch_ms"], "ms")' 2>/dev/null)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
