#!/bin/bash
# round-3 GPU check: the whole -m gpu suite, then the C2 bench with and without
# the per-iteration output files.  Every GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --write --no-cpu-baseline \
    > gpurun_out/${tag}_bench_c2.json 2> gpurun_out/${tag}_bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench_c2.err; exit 1; }
cat gpurun_out/${tag}_bench_c2.json
