#!/bin/bash
# C2 default bench line (with both CPU legs) and the C3 shard line.
#   gpurun --timeout 900 -- bash tools/gpu_bench2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2_ref.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_c2_ref.log
timeout -k 10 400 python bench.py --config c3 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_c3.log
