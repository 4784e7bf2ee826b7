#!/bin/bash
# The head-start kernel's plan at the C3 shard (configuration 8 at S = 4
# instead of 9): old build (build_old/lib) vs the tree's build, one box.
#   1. bitwise: 12 linear iterations at N = 100,000 (team of 32, S = 4);
#   2. the head-start / one-pass / scale GPU tests on the new build;
#   3. the C3 shard bench alternating old / new, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03h}
OLD=$PWD/build_old/lib/libvampomi.so
NEW=$PWD/vampomi_amd/lib/libvampomi.so
for b in old new; do
  lib=$OLD; [ $b = new ] && lib=$NEW
  VAMPOMI_LIB=$lib timeout -k 10 180 python -u tools/lib_bitwise.py run gpurun_out/${tag}_$b.npz 100000 20000 12 linear \
    > gpurun_out/${tag}_bitwise_$b.log 2>&1 || { echo "run $b failed"; tail -5 gpurun_out/${tag}_bitwise_$b.log; exit 1; }
done
python tools/lib_bitwise.py cmp gpurun_out/${tag}_old.npz gpurun_out/${tag}_new.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_operator.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for rep in 1 2; do
  for b in old new; do
    lib=$OLD; [ $b = new ] && lib=$NEW
    VAMPOMI_LIB=$lib timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${tag}_c3_$b$rep.json 2>> gpurun_out/${tag}.err || { echo "bench $b failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_c3_$b$rep.json') if l.startswith('{')][-1]); r=d['roofline']; print('$b$rep', d['value'], d['ms_per_step'], d['passes_exec_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
  done
done
