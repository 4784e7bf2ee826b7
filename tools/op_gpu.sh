#!/bin/bash
# one-pass operator bring-up: its GPU parity tests, kernel variants, C2 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k onepass -x -v -s -rf --timeout 120 --timeout-method thread > gpurun_out/op_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|onepass vs" gpurun_out/op_pytest.log | head -30; tail -5 gpurun_out/op_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kbench.py 10000 50000 10 op,atx > gpurun_out/op_kbench.log 2>&1; rc=$?
echo "kbench rc=$rc"; grep -E "^op|^atx" gpurun_out/op_kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --batch-rhs 4 --no-cpu-baseline > gpurun_out/op_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/op_bench.log | cut -c1-700
exit $rc
