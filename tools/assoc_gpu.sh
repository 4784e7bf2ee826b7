#!/bin/bash
# gpurun session for the association-test row: its GPU tests, the c5 bench
# line, a rocprofv3 kernel trace and the PMC traffic pass.
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
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
step assoc_tests 600 python -m pytest tests/test_gpu_assoc.py -q -rf
step bench_c5 400 python bench.py --config c5 --steps 10 --warmup 2
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline
step pmc_c5 500 bash tools/pmc.sh c5
echo done
