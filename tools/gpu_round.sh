#!/bin/bash
# The measurement round in two gpurun sessions (each GPU step has its own time
# limit; the script stops at the first abnormal exit, i.e. not 0 / 1):
#   part a: smoke, the GPU tests, C2 (default bench line with CPU baseline,
#           rocprofv3 kernel stats, PMC traffic), config-4 probit shard (same)
#   part b: C5 association shard (same), ingest, the C3 shard, config 4 whole
#           and 240 GB on one GPU (c3big)
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh a|b
set -u
PART=${1:-a}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
prof() {  # workload steps
    step "rocprof_$1" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$1" -o run --output-format csv -- \
        python bench.py --config "$1" --steps "$2" --warmup 2 --no-cpu-baseline
}
if [ "$PART" = a ]; then
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
    step bench_c2 400 python bench.py
    prof c2 20
    step pmc_c2 400 bash tools/pmc.sh c2
    step bench_c4 500 python bench.py --config c4 --steps 12 --warmup 2
    prof c4 6
    step pmc_c4 500 bash tools/pmc.sh c4
else
    step bench_c5 400 python bench.py --config c5 --steps 10 --warmup 2
    prof c5 6
    step pmc_c5 500 bash tools/pmc.sh c5
    step ingest 600 python tools/ingest_bench.py 100000 25000
    step bench_c3 900 python bench.py --config c3 --steps 10 --warmup 2
    prof c3 4
    step bench_c4full 600 python bench.py --config c4full --steps 6 --warmup 2 --no-cpu-baseline
    step bench_c3big 600 python bench.py --config c3big --steps 4 --warmup 1
fi
echo "done"
