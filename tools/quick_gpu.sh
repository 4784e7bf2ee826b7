#!/bin/bash
# quick gpurun check: the GPU test suite, then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_c2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-timing > gpurun_out/bench_c2_nt.log 2>&1; rc=$?
echo "bench (no timing) rc=$rc"; tail -1 gpurun_out/bench_c2_nt.log
exit $rc
