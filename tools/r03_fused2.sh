#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03k}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fused or onepass" tests/test_gpu_operator.py > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
VAMPOMI_LIB=$PWD/build_ts/lib/libvampomi.so VAMPOMI_TAIL_TS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing > gpurun_out/${tag}_ts.json 2> gpurun_out/${tag}_ts.err || { echo ts failed; tail gpurun_out/${tag}_ts.err; exit 1; }
grep "fused tail" gpurun_out/${tag}_ts.err
for f in 1 0 1 0; do
  VAMPOMI_OP_FUSED=$f timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_f$f.json 2>> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_f$f.json')); r=d['roofline']; print('fused=$f', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'], d['cg_iters'][-3:])"
done
