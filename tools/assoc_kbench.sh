#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_assoc.py -q -rf > gpurun_out/assoc_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -25 gpurun_out/assoc_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/kbench.py 100000 62500 10 loo > gpurun_out/kbench_loo.log 2>&1; rc=$?
echo "kbench rc=$rc"; grep "^loo" gpurun_out/kbench_loo.log
