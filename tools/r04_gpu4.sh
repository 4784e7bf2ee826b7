#!/bin/bash
# Round 4: the GPU suite on this build, bitwise and rate A/B against
# build_old, and a kernel trace of the default C2 line (gap analysis).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=$PWD/build_old/lib/libvampomi.so
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
brief() { grep '^{' "$OUT/$1.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"; }
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for m in linear bin_class; do
    step bw_new_$m 200 python tools/lib_bitwise.py run "$OUT/new_$m.npz" 10000 20000 12 $m
    step bw_old_$m 200 env VAMPOMI_LIB=$OLD python tools/lib_bitwise.py run "$OUT/old_$m.npz" 10000 20000 12 $m
    python tools/lib_bitwise.py cmp "$OUT/new_$m.npz" "$OUT/old_$m.npz" | tee -a "$OUT/bitwise.txt"
done
for r in 1 2 3; do
    step ab_new_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline && brief ab_new_$r | tee -a "$OUT/ab.txt"
    step ab_old_$r 200 env VAMPOMI_LIB=$OLD python bench.py --steps 20 --warmup 5 --no-cpu-baseline && brief ab_old_$r | tee -a "$OUT/ab.txt"
done
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline
f=$(find "$OUT/prof" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_gaps.py "$f" 0.3 > "$OUT/gaps.txt" && head -34 "$OUT/gaps.txt"
echo done
