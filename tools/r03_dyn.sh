#!/bin/bash
# dynamic chunks: operator tests, VAMP parity on dyn plans, the skew of a dyn
# launch (TM_TS build), then the C2 bench static (1407 = the default plan) /
# dyn (1417), twice.  One box; every GPU step time-limited; stops at a failure.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_operator.py tests/test_gpu_parity.py -m gpu -x -v -k "dynamic_chunks_vamp" \
    --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/${tag}_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_tests.log | tail -25
VAMPOMI_LIB=$PWD/vampomi_amd/lib_ts/libvampomi.so VAMPOMI_OP_TS=1 timeout -k 10 120 python -u tools/op_skew.py 10000 50000 6 2 1417 \
    > gpurun_out/${tag}_skew_c2_dyn.txt 2>&1 || { echo skew failed; tail -20 gpurun_out/${tag}_skew_c2_dyn.txt; exit 1; }
cut -c1-330 gpurun_out/${tag}_skew_c2_dyn.txt
for rep in 1 2; do
  for v in 1407 1417; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --op-variant $v \
        > gpurun_out/${tag}_bench_c2_v$v.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['passes_exec_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['a_kernel_frac_of_step'])" gpurun_out/${tag}_bench_c2_v$v.json v=$v
  done
done
