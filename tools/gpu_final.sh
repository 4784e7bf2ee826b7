#!/bin/bash
# Round-end evidence for the current build: smoke, the default C2 bench line
# (both CPU legs), its rocprofv3 kernel stats and PMC traffic; the same for the
# C3 shard and the config-4 probit shard.
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
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
prof() {
    step "rocprof_$1" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$1" -o run --output-format csv -- \
        python bench.py --config "$1" --steps "$2" --warmup 5 --no-cpu-baseline
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 400 python bench.py --steps 20 --warmup 5
prof c2 20
step pmc_c2 300 bash tools/pmc.sh c2
step bench_c3 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline
prof c3 6
step pmc_c3 300 bash tools/pmc.sh c3
step bench_c4 300 python bench.py --config c4 --steps 12 --warmup 2 --no-cpu-baseline
prof c4 8
echo done
