#!/bin/bash
# bench with and without the live kernel timing, and the rocprofv3 --stats
# summary of the timed command (its average for the roofline kernel must agree)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_t.log 2>&1 || exit $?
tail -1 gpurun_out/bench_t.log | cut -c1-900
timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing > gpurun_out/bench_nt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_nt.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_t.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_t.log | cut -c1-900
head -4 gpurun_out/prof_t/run_kernel_stats.csv | cut -c1-160
