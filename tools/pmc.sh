#!/bin/bash
# HBM traffic of the A / A^T kernels from PMC counters (MI355X_MICROARCH.md
# §HBM): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not
# fit one pass), kernel dispatch rows only, no tracing domains.
#   gpurun -- bash tools/pmc.sh [config]      (bench.py --config, default c2)
set -u
CFG=${1:-c2}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$CFG
mkdir -p "$OUT"
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc "$C" -d "$OUT/$C" -o run --output-format csv -- \
        python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-timing > "$OUT/$C.log" 2>&1 || exit $?
done
python tools/pmc_parse.py "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
