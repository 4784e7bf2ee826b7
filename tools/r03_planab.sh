#!/bin/bash
# C2 operator plans in VAMP, alternating, three rounds (bench.py --op-variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03pl}
plans=${2:--1 1212 48}
for rep in 1 2 3; do
  for v in $plans; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --op-variant $v > gpurun_out/${tag}_v${v}_$rep.json 2>> gpurun_out/${tag}.err || { echo "bench $v failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_v${v}_$rep.json') if l.startswith('{')][-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
  done
done
