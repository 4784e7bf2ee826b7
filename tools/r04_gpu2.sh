#!/bin/bash
# Round 4, second call: rank 0's 1-GPU bases outside a job, the 2-rank launcher
# on one GPU again (its expected RCCL refusal, now after the bases), and the
# C3 / C5 shard lines with the reference's own operators timed on a sub-shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 3 "$OUT/$name.log" | cut -c1-600
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step bases 200 python tools/r04_bases.py
step bench_c3 400 python bench.py --config c3 --steps 10 --warmup 2
step bench_c5 300 python bench.py --config c5 --steps 5 --warmup 1
echo "== spawn2_on_one_gpu ($(date +%T))"
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --deadline-s 240 > "$OUT/spawn2.log" 2>&1
echo "rc=$?" >> "$OUT/spawn2.log"
tail -n 2 "$OUT/spawn2.log" | cut -c1-2500
echo done
