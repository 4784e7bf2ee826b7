#!/bin/bash
# Round 4: the whole-shard oracle parity tests (C3, C5), then r04_gpu5.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04j
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py::test_c3_full_shard_vs_oracle \
    tests/test_gpu_assoc.py::test_c5_full_shard_vs_oracle -m gpu -v --durations=0 --timeout 300 \
    --timeout-method thread > "$OUT/fullshard.log" 2>&1
rc=$?
tail -15 "$OUT/fullshard.log"
[ $rc -eq 0 ] || exit $rc
bash tools/r04_gpu5.sh r04h
