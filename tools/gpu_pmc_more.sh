#!/bin/bash
# PMC traffic of the probit shard (merged first launch), config 4 whole and
# the 240 GB shape, and the 240 GB rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c4 c4full c3big; do
    timeout -k 10 400 bash tools/pmc.sh $w > gpurun_out/pmc_$w.log 2>&1 || { tail gpurun_out/pmc_$w.log; exit 1; }
    echo "pmc $w ok"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3big -o run --output-format csv -- \
    python bench.py --config c3big --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rocprof_c3big.log 2>&1 || exit 1
echo done
