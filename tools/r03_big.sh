#!/bin/bash
# Round-3 lines of the larger workloads on one box (the head start on by
# default): the C3 shard and the config-4 probit shard (bench line with the
# CPU leg, rocprofv3 kernel stats, PMC traffic), config 4 whole, 240 GB on one
# GPU (c3big) and the C5 LOO shard.  Stops at the first abnormal exit.
#   gpurun --timeout 1200 -- bash tools/r03_big.sh
set -u
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
    grep '^{' "$OUT/$name.log" | tail -n 1 | cut -c1-300
    if [ $rc -ne 0 ]; then
        tail -n 5 "$OUT/$name.log"
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
prof() {  # workload steps
    step "rocprof_$1" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$1" -o run --output-format csv -- \
        python bench.py --config "$1" --steps "$2" --warmup 2 --no-cpu-baseline
}
step bench_c3 400 python bench.py --config c3 --steps 10 --warmup 2
prof c3 6
step pmc_c3 300 bash tools/pmc.sh c3
step bench_c4 300 python bench.py --config c4 --steps 12 --warmup 2
prof c4 8
step bench_c4full 300 python bench.py --config c4full --steps 6 --warmup 2 --no-cpu-baseline
step bench_c3big 400 python bench.py --config c3big --steps 4 --warmup 1
step bench_c5 300 python bench.py --config c5 --steps 10 --warmup 2
echo done
