#!/bin/bash
# rocprofv3 kernel trace + stats of the default C2 bench, then the PMC traffic passes
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=${1:-c2}; STEPS=${2:-20}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- \
    python bench.py --config $CFG --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_$CFG.log 2>&1 || exit $?
tail -1 gpurun_out/rocprof_$CFG.log
bash tools/pmc.sh $CFG
