#!/bin/bash
# fused CG tail timing experiments (TAIL_EXP builds in build_exp<k>/, results wrong there), all on one box
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03h}
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_$name.json')); r=d['roofline']; print('%-10s' % '$name', d['value'], d['ms_per_step'], r['avg_launch_us'], d['a_kernel_frac_of_step'])"
}
for rep in 1 2; do
  run unfused$rep VAMPOMI_OP_FUSED=0
  run fused$rep VAMPOMI_OP_FUSED=1
  run plaind$rep VAMPOMI_LIB=$PWD/build_exp1/lib/libvampomi.so
  run noupd$rep VAMPOMI_LIB=$PWD/build_exp2/lib/libvampomi.so
  run nobar$rep VAMPOMI_LIB=$PWD/build_exp3/lib/libvampomi.so
done
