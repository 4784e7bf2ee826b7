#!/bin/bash
# C5 evidence for the LOO pass default: the whole -m gpu suite, the C5 bench
# line (CPU leg on), its rocprofv3 kernel stats and PMC traffic.
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
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step bench_c5 400 python bench.py --config c5 --steps 10 --warmup 2
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- \
    python bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline
step pmc_c5 300 bash tools/pmc.sh c5
echo done
