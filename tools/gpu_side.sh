#!/bin/bash
# Side-stream check: its GPU tests, the whole GPU suite, a C2 A/B of one
# stream against two (VAMPOMI_SIDE_STREAM), and a kernel trace whose
# em/denoise kernels are checked for overlap with the main stream's kernels.
#   gpurun --timeout 900 -- bash tools/gpu_side.sh
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
    tail -n 3 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
step side_tests 300 python -u -m pytest tests/test_gpu_sharded.py -m gpu -v -rf --timeout 120 --timeout-method thread -k side_stream
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for k in 1 2; do
    for s in 0 1; do
        VAMPOMI_SIDE_STREAM=$s step "ab_c2_side${s}_$k" 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline
    done
done
step trace_c2 300 rocprofv3 --kernel-trace -d "$OUT/trace_c2" -o run --output-format csv -- \
    python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline
for f in "$OUT"/trace_c2/*kernel_trace.csv; do
    python tools/trace_overlap.py "$f" "$OUT/side_overlap_c2.json"
done
echo done
