#!/bin/bash
# Sampled timing (bench.py --timing-period 4, hashed positions) against every
# launch timed and no timing, alternating on one box; then rocprofv3 of the
# default command: its operator average and A-kernel total against the line's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03tp}
run() {  # name extra-args...
  local name=$1; shift
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); r=d['roofline'] or {}; print('%-6s' % '$name', d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('timed_launches'), r.get('frac'), d['a_kernel_frac_of_step'])"
}
for rep in 1 2 3; do
  run p4_$rep
  run p1_$rep --timing-period 1
  run nt_$rep --no-timing
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/kstats.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_prof_real.csv
grep '^{' gpurun_out/${tag}_prof.log | tail -1 > gpurun_out/${tag}_prof_line.json
python3 - gpurun_out/${tag}_prof_real.csv gpurun_out/${tag}_prof_line.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
a_ns = sum(float(r["TotalDurationNs"]) for r in rows if any(k in r["Name"] for k in ("atax_", "ax_partial", "atx_kernel")))
op = [r for r in rows if "atax_team_kernel<2" in r["Name"]][0]
real = int(op["Calls"]) - int(op["GatedCalls"])
print("rocprof: operator avg (real launches) %.1f us; A-kernel total %.2f ms" % (float(op["TotalDurationNs"]) / max(real, 1) / 1e3 if False else float(op["AverageNs"]) / 1e3, a_ns / 1e6))
print("line: operator avg %.1f us; a_kernel_frac %.4f x %.3f ms x %d steps = %.2f ms" % (d["roofline"]["avg_launch_us"], d["a_kernel_frac_of_step"], d["ms_per_step"], d["steps"], d["a_kernel_frac_of_step"] * d["ms_per_step"] * d["steps"]))
PY
