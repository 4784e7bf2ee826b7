#!/bin/bash
# Round 4, third call: the probit bar's gap / spread ratios; bitwise and rate
# A/B of this build against build_old (cg_update per system count, 32 slot
# loads in flight); the C2 operator's workgroup skew for the default team of 2
# (TM_TS build) and for T = 1; the two plans in VAMP; a kernel trace of the
# default C2 line for the gap analysis (tools/trace_gaps.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04c
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=$PWD/build_old/lib/libvampomi.so
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 3 "$OUT/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
brief() { grep '^{' "$OUT/$1.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"; }
for m in linear bin_class; do
    step bw_new_$m 200 python tools/lib_bitwise.py run "$OUT/new_$m.npz" 10000 20000 12 $m
    step bw_old_$m 200 env VAMPOMI_LIB=$OLD python tools/lib_bitwise.py run "$OUT/old_$m.npz" 10000 20000 12 $m
    python tools/lib_bitwise.py cmp "$OUT/new_$m.npz" "$OUT/old_$m.npz"
done
for r in 1 2 3; do
    step ab_new_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline && brief ab_new_$r
    step ab_old_$r 200 env VAMPOMI_LIB=$OLD python bench.py --steps 20 --warmup 5 --no-cpu-baseline && brief ab_old_$r
done
for r in 1 2; do
    step ab_t1_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --op-variant 10 && brief ab_t1_$r
done
step skew_t2 120 env VAMPOMI_LIB=$PWD/vampomi_amd/lib_ts/libvampomi.so VAMPOMI_OP_TS=1 python -u tools/op_skew.py 10000 50000 6 2
step skew_t1 120 env VAMPOMI_LIB=$PWD/vampomi_amd/lib_ts/libvampomi.so VAMPOMI_OP_TS=1 python -u tools/op_skew.py 10000 50000 6 2 10
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline
f=$(find "$OUT/prof" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_gaps.py "$f" 0.3 > "$OUT/gaps.txt" && head -32 "$OUT/gaps.txt"
bash tools/r04_probit_k.sh
echo done
