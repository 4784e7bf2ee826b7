#!/bin/bash
# the fused CG tail: its parity tests, the C2 bench with and without it, and a
# kernel trace of each (tools/trace_op.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03g}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fused or onepass" tests/test_gpu_operator.py > gpurun_out/${tag}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for f in 1 0 1 0; do
  VAMPOMI_OP_FUSED=$f timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_f$f.json 2>> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_f$f.json')); r=d['roofline']; print('fused=$f', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'], d['cg_iters'][-3:])"
done
for f in 1 0; do
  VAMPOMI_OP_FUSED=$f timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${tag}_prof_f$f -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing > /dev/null 2>> gpurun_out/${tag}_bench.err || { echo "prof failed"; exit 1; }
  echo "== fused=$f"
  python tools/trace_op.py $(find gpurun_out/${tag}_prof_f$f -name "*kernel_trace.csv" | head -1) | head -4
  python tools/trace_gaps.py $(find gpurun_out/${tag}_prof_f$f -name "*kernel_trace.csv" | head -1) 0.3 | head -4
done
