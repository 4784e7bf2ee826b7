#!/bin/bash
# Round 4, first GPU call: the GPU suite, the default C2 line, the C2 line over
# a 1-rank RCCL communicator (the non-blocking creation and collectives), and
# the 2-rank launcher on a 1-GPU box (rank 0's 1-GPU bases run; RCCL then
# refuses two ranks on one GPU, which must end in ONE failure line, rc != 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04a
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 3 "$OUT/$name.log" | cut -c1-400
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
step gputests 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_c2 300 python bench.py --steps 20 --warmup 5
step bench_c2_rccl1 200 env VAMPOMI_FORCE_RCCL=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo "== spawn2_on_one_gpu ($(date +%T))"
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --deadline-s 240 > "$OUT/spawn2.log" 2>&1
echo "rc=$?" >> "$OUT/spawn2.log"
tail -n 4 "$OUT/spawn2.log" | cut -c1-1500
echo done
