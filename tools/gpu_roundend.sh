#!/bin/bash
# Round-end check of the tree as the driver runs it (smoke, the GPU suite,
# the default bench line), stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { tail gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log | cut -c1-400
