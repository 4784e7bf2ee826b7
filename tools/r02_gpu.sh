#!/bin/bash
# Round-2 GPU session: each GPU step under its own time limit; the script
# stops at the first abnormal exit (not 0 / 1).
#   gpurun --timeout 1200 -- bash tools/r02_gpu.sh <steps...>
#   steps: smoke tests tests:<pytest -k expr> bench:<config>:<steps> prof:<config>:<steps> pmc:<config>
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
    tail -n 4 "$OUT/$name.log" | cut -c1-600
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
for s in "$@"; do
    IFS=: read -r kind a b <<< "$s"
    case $kind in
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread ;;
        tests1) step "pytest_$a" 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread -k "$a" ;;
        bench) step "bench_$a" 900 python bench.py --config "$a" --steps "${b:-20}" --warmup 5 ;;
        benchn) step "bench_${a}_nocpu" 900 python bench.py --config "$a" --steps "${b:-20}" --warmup 5 --no-cpu-baseline ;;
        prof) step "rocprof_$a" 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a" -o run --output-format csv -- \
                  python bench.py --config "$a" --steps "${b:-10}" --warmup 2 --no-cpu-baseline ;;
        pmc) step "pmc_$a" 500 bash tools/pmc.sh "$a" ;;
        pmcsq) step "pmcsq_$a" 300 bash tools/pmc_sq.sh "$a" ;;
        kbench) step "kbench_$a" 600 python tools/kbench.py $a ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "done"
