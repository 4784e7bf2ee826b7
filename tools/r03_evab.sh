#!/bin/bash
# Timing-event fence A/B at C2: old build (default events) / new build
# (hipEventDisableSystemFence), each with the bench's HIP-event timing on and
# off, alternating on one box; plus the new build's kernel timing against
# rocprofv3 of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03t}
OLD=$PWD/build_old/lib/libvampomi.so
NEW=$PWD/vampomi_amd/lib/libvampomi.so
run() {  # name lib extra-args...
  local name=$1 lib=$2; shift 2
  VAMPOMI_LIB=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); r=d['roofline'] or {}; print('%-12s' % '$name', d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), d['a_kernel_frac_of_step'])"
}
for rep in 1 2; do
  run old_t$rep "$OLD"
  run new_t$rep "$NEW"
  run old_n$rep "$OLD" --no-timing
  run new_n$rep "$NEW" --no-timing
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/kstats.py gpurun_out/${tag}_prof/run_kernel_trace.csv | grep atax_team_kernel | cut -c1-60,150-
grep '^{' gpurun_out/${tag}_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('events', d['roofline']['avg_launch_us'], d['a_kernel_frac_of_step'])"
