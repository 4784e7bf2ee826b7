#!/bin/bash
# round-3: the CG head start.  Head-start GPU tests first, then the whole -m gpu
# suite, then the C2 bench with the head start on / off / on (one box).  Every
# GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03hs}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "headstart or onepass" --timeout 240 \
    --timeout-method thread > gpurun_out/${tag}_hs_tests.log 2>&1 || { echo "head-start tests failed"; tail -60 gpurun_out/${tag}_hs_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_hs_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_gpu_tests.log
for hs in 1 0 1; do
  VAMPOMI_HEADSTART=$hs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${tag}_bench_c2_hs$hs.json 2> gpurun_out/${tag}_bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench_c2.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['passes_exec_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['a_kernel_frac_of_step'])" gpurun_out/${tag}_bench_c2_hs$hs.json hs=$hs
done
