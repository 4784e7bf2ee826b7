#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03p}
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env VAMPOMI_LIB=$lib "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_$name.json')); r=d['roofline']; print('%-12s' % '$name', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
}
L=$PWD/vampomi_amd/lib/libvampomi.so; X=$PWD/build_xp0/lib/libvampomi.so
for rep in 1 2; do
  run nt_fwd$rep $L
  run nt_alt$rep $L VAMPOMI_OP_ALT=1
  run def_fwd$rep $X
  run def_alt$rep $X VAMPOMI_OP_ALT=1
done
OP_PLANS=-1 VAMPOMI_OP_ALT=1 timeout -k 10 120 python tools/kbench.py 10000 50000 20 op 2>&1 | grep '^op' | sed 's/^/alt standalone nt: /'
OP_PLANS=-1 VAMPOMI_LIB=$X VAMPOMI_OP_ALT=1 timeout -k 10 120 python tools/kbench.py 10000 50000 20 op 2>&1 | grep '^op' | sed 's/^/alt standalone def: /'
OP_PLANS=-1 VAMPOMI_LIB=$X timeout -k 10 120 python tools/kbench.py 10000 50000 20 op 2>&1 | grep '^op' | sed 's/^/fwd standalone def: /'
