#!/bin/bash
# Round-2 operator session: the operator parity test, then the plan sweep at
# C2 and at the C3 shard; stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
run() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 6 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
    IFS=: read -r kind a b c <<< "$s"
    case $kind in
        optest) run optest 600 python -u -m pytest tests/test_gpu_operator.py -x -v -rf --timeout 300 --timeout-method thread ;;
        tests1) run "pytest_$a" 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "$a" ;;
        kb) run "kbench_op_${a}_${b}" 600 python tools/kbench.py "$a" "$b" "${c:-10}" op ;;
        # team plans honour VAMPOMI_OP_DBG only in a TM_DBG=1 build: DBGLIB=<that .so> (vampomi_amd/csrc/Makefile)
        kbdbg) [ -n "${DBGLIB:-}" ] && export VAMPOMI_LIB="$DBGLIB"; for dbg in ${DBGS:-0 1 2 3 4 8 15}; do VAMPOMI_OP_DBG=$dbg OP_PLANS=$c run "kbench_dbg${dbg}_${a}_${b}" 300 python tools/kbench.py "$a" "$b" 5 op; done ;;
        bench) run "bench_$a" 900 python bench.py --config "$a" --steps "${b:-20}" --warmup 5 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo done
