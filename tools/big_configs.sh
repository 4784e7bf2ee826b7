#!/bin/bash
# one-GPU bench lines for the big BASELINE shapes: the C3 shard (50 GB,
# methylation-like; 8 of them = N=100k x Mt=500k) and configs[3] whole (80 GB)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log
timeout -k 10 600 python bench.py --config c4full --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4full.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit $?
head -5 gpurun_out/prof_c3/run_kernel_stats.csv | cut -c1-140
