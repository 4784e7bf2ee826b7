#!/bin/bash
# Final round-3 evidence of the current build on one box: smoke, the whole
# -m gpu suite, the default C2 bench line (both CPU legs), its rocprofv3
# kernel stats and PMC traffic, and the config-4 probit shard line + stats.
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
    grep '^{' "$OUT/$name.log" | tail -n 1 | cut -c1-200
    tail -n 1 "$OUT/$name.log" | cut -c1-200
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step bench_c2 400 python bench.py
step rocprof_c2 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- \
    python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline
step pmc_c2 300 bash tools/pmc.sh c2
step bench_c4 300 python bench.py --config c4 --steps 12 --warmup 2
step rocprof_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
    python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline
step pmc_c4 300 bash tools/pmc.sh c4
echo done
