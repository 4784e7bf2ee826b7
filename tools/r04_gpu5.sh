#!/bin/bash
# Round 4: what the sampled HIP-event timing costs the C2 rate (period 4 / 16 /
# none, alternating), and a HIP API + kernel trace of the default C2 line (the
# host's time between a flag and its next launches).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-r04h}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; }
}
brief() { grep '^{' "$OUT/$1.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$1', d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('timed_launches'), d['a_kernel_frac_of_step'])" | tee -a "$OUT/timing_ab.txt"; }
for r in 1 2 3; do
    step tp4_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timing-period 4 && brief tp4_$r
    step tp16_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timing-period 16 && brief tp16_$r
    step tpnone_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing && brief tpnone_$r
done
step hiptrace 300 rocprofv3 --hip-trace --kernel-trace -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --steps 6 --warmup 2 --no-cpu-baseline
ls -R "$OUT/prof" | head -20
echo done
