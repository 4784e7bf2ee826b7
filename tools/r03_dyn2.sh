#!/bin/bash
# dynamic chunks, second form: probe on the TM_SAFE build, then the dyn tests,
# the skew of a dyn launch and the C2 bench static / dyn.  Stops at a failure.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03e}
VAMPOMI_LIB=$PWD/vampomi_amd/lib_safe/libvampomi.so timeout -k 10 240 python -u tools/op_plan_probe.py 1000 3000 1217 1218 1417 1418 1817 1818 \
    > gpurun_out/${tag}_probe.txt 2>&1 || { echo probe failed; cat gpurun_out/${tag}_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_probe.txt | tail -4
bash tools/r03_dyn.sh $tag
