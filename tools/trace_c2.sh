#!/bin/bash
# C2 GPU tests (parity), then a kernel trace of a short bench without event timing
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_probit.py tests/test_gpu_sharded.py -q -x > gpurun_out/pytest_core.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_core.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-timing > gpurun_out/bench_nt.log 2>&1; rc=$?
echo "bench no-timing rc=$rc"; tail -1 gpurun_out/bench_nt.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/prof3.log 2>&1; rc=$?
echo "trace rc=$rc"
exit $rc
