#!/bin/bash
# Probit with the merged first launch: its GPU tests, the whole suite, and
# the config-4 bench lines (shard, whole) with a rocprofv3 kernel-stats run.
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
    tail -n 3 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step probit_tests 400 python -u -m pytest tests/test_gpu_probit.py tests/test_gpu_sharded.py -m gpu -v -rf --timeout 120 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step bench_c4 300 python bench.py --config c4 --steps 12 --warmup 2
step bench_c4full 400 python bench.py --config c4full --steps 6 --warmup 2 --no-cpu-baseline
step rocprof_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4p" -o run --output-format csv -- \
    python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline
echo done
