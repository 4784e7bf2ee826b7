#!/bin/bash
# A/B of library builds on one box: VAMPOMI_LIB=<lib> bench.py (C2), alternating
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03n}
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env VAMPOMI_LIB=$lib "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_$name.json')); r=d['roofline']; print('%-12s' % '$name', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
}
for rep in 1 2 3; do
  run old$rep $PWD/build_old/lib/libvampomi.so
  run new$rep $PWD/vampomi_amd/lib/libvampomi.so
done
