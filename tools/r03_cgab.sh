#!/bin/bash
# A library change that must not move a bit (e.g. the cg_update latency
# rework): old build (build_old/lib) vs the tree's build on one box.
#   1. the same VAMP runs (linear C2 window shape, probit) with each build, compared bitwise;
#   2. the whole -m gpu suite on the new build;
#   3. the C2 bench alternating old / new, three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
tag=${1:-r03c}
OLD=$PWD/build_old/lib/libvampomi.so
NEW=$PWD/vampomi_amd/lib/libvampomi.so
for m in linear bin_class; do
  for b in old new; do
    lib=$OLD; [ $b = new ] && lib=$NEW
    VAMPOMI_LIB=$lib timeout -k 10 120 python -u tools/lib_bitwise.py run gpurun_out/${tag}_${m}_$b.npz 10000 20000 12 $m \
      > gpurun_out/${tag}_bitwise_${m}_$b.log 2>&1 || { echo "run $m $b failed"; tail -5 gpurun_out/${tag}_bitwise_${m}_$b.log; exit 1; }
  done
  python tools/lib_bitwise.py cmp gpurun_out/${tag}_${m}_old.npz gpurun_out/${tag}_${m}_new.npz
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
run() {  # name lib
  local name=$1 lib=$2
  VAMPOMI_LIB=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_$name.json 2>> gpurun_out/${tag}.err || { echo "$name failed"; tail -5 gpurun_out/${tag}.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${tag}_$name.json') if l.startswith('{')][-1]); r=d['roofline']; print('%-6s' % '$name', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['a_kernel_frac_of_step'])"
}
for rep in 1 2 3; do
  run old$rep "$OLD"
  run new$rep "$NEW"
done
# the operator alone (tools/kbench.py op, default plan), old / new / old / new
for rep in 1 2; do
  for b in old new; do
    lib=$OLD; [ $b = new ] && lib=$NEW
    VAMPOMI_LIB=$lib OP_PLANS=-1 timeout -k 10 120 python -u tools/kbench.py 10000 50000 20 op > gpurun_out/${tag}_kb_$b$rep.txt 2>&1 || { echo "kbench $b failed"; exit 1; }
    echo "kbench $b$rep $(grep '^op ' gpurun_out/${tag}_kb_$b$rep.txt | cut -c1-160)"
  done
done
