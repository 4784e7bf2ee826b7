#!/bin/bash
# Round-3 evidence on one box, stopping at the first abnormal exit:
#   smoke, the whole -m gpu suite, the default C2 bench line (both CPU legs),
#   its rocprofv3 kernel stats and PMC traffic, then the C2 operator plans
#   named in $1 in VAMP (bench.py --op-variant, default plan first and last).
#   gpurun --timeout 1200 -- bash tools/r03_evidence.sh [plans]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
plans=${1:-}
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
step bench_c2 400 python bench.py --steps 20 --warmup 5
step rocprof_c2 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- \
    python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline
step pmc_c2 400 bash tools/pmc.sh c2
for v in $plans; do
    step "bench_c2_v$v" 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --op-variant "$v"
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])" "$OUT/bench_c2_v$v.log" "$v"
done
echo done
