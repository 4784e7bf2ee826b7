#!/bin/bash
# One gpurun session covering every bench workload: smoke, the GPU tests,
# bench lines (c2 default, c4 probit, c5 association) with CPU baselines, a
# rocprofv3 kernel trace and the PMC traffic pass per extra workload.  Each GPU step has its
# own time limit; the script stops at the first abnormal exit (not 0 / 1).
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh
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
    tail -n 4 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
step bench_c2 400 python bench.py
step bench_c4 500 python bench.py --config c4 --steps 12 --warmup 2
step rocprof_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline
step pmc_c4 500 bash tools/pmc.sh c4
step bench_c5 400 python bench.py --config c5 --steps 10 --warmup 2
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline
step pmc_c5 500 bash tools/pmc.sh c5
step ingest 600 python tools/ingest_bench.py 100000 25000
echo "done"
