#!/bin/bash
# C2 one-pass operator plans: standalone sweep (tools/kbench.py) and in VAMP
# (bench.py --op-variant), plus the bench's timing on/off, all on one box.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03b}
plans=${2:--1,1210,1211,1212,1410,1412,48,49}
OP_PLANS=$plans timeout -k 10 300 python -u tools/kbench.py 10000 50000 20 op > gpurun_out/${tag}_kbench_op.txt 2>&1 || { tail -20 gpurun_out/${tag}_kbench_op.txt; exit 1; }
grep '^op' gpurun_out/${tag}_kbench_op.txt
for v in ${plans//,/ }; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --op-variant $v > gpurun_out/${tag}_bench_v$v.json 2>> gpurun_out/${tag}_bench.err || { echo "bench $v failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${tag}_bench_v$v.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing > gpurun_out/${tag}_bench_notiming.json 2>> gpurun_out/${tag}_bench.err && python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_notiming.json')); print('no-timing', d['value'], d['ms_per_step'])"
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_default2.json 2>> gpurun_out/${tag}_bench.err && python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_default2.json')); print('default again', d['value'], d['ms_per_step'])"
