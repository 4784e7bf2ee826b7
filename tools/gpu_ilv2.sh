#!/bin/bash
# Interleaved team columns as the default: the remaining team shapes A/B,
# the GPU suite, and the bench lines of every linear/probit workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
run() {  # name timeout cmd...
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
OP_PLANS=46,47,46,47 run ilv_c2 200 python tools/kbench.py 10000 50000 20 op
grep '^op' "$OUT/ilv_c2.log"
OP_PLANS=166,167,166,167 run ilv_c4 200 python tools/kbench.py 50000 50000 10 op
grep '^op' "$OUT/ilv_c4.log"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run bench_c2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_c3 400 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline
run bench_c4 300 python bench.py --config c4 --steps 12 --warmup 2 --no-cpu-baseline
run bench_c4full 400 python bench.py --config c4full --steps 6 --warmup 2 --no-cpu-baseline
run bench_c3big 500 python bench.py --config c3big --steps 4 --warmup 1 --no-cpu-baseline
echo done
