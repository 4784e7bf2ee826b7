#!/bin/bash
# kernel trace of the C2 bench without the live HIP-event timing (gap analysis)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_nt -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/prof_nt.log 2>&1 || exit $?
python tools/trace_gaps.py gpurun_out/prof_nt/run_kernel_trace.csv > gpurun_out/prof_nt_gaps.txt
