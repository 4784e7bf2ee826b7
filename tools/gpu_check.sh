#!/bin/bash
# One gpurun session: smoke, GPU tests, a short bench and a rocprofv3 kernel
# trace.  Every GPU step has its own time limit; the script stops at the first
# step that dies abnormally (anything other than exit 0 or an ordinary test
# failure, exit 1).
#   gpurun --timeout 1200 -- bash tools/gpu_check.sh [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${1:-10}
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 8 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
(rocminfo | grep -m2 -E "gfx|Marketing" ; nproc; free -g | head -2) > "$OUT/host.txt" 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -m gpu -q -rf
step bench 600 python bench.py --steps "$STEPS" --warmup 2
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline
echo "done"
