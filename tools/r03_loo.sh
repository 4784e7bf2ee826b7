#!/bin/bash
# LOO pass variants: the association GPU tests, then the standalone sweep at
# the C5 shard (tools/kbench.py loo) and the C5 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_assoc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u tools/kbench.py 100000 62500 10 loo > gpurun_out/${tag}_kbench_loo.txt 2>&1 || { echo "kbench failed"; tail -5 gpurun_out/${tag}_kbench_loo.txt; exit 1; }
grep '^loo' gpurun_out/${tag}_kbench_loo.txt | cut -c1-140
