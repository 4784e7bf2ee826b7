#!/bin/bash
# diagnostic: every operator plan at N=1000 x 3000 one launch at a time, on the
# TM_SAFE build (columns outside the shard are reported, not read)
set -o pipefail
mkdir -p gpurun_out
VAMPOMI_LIB=$PWD/vampomi_amd/lib_safe/libvampomi.so AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 python -u tools/op_plan_probe.py 1000 3000 \
    1217 1218 1417 1418 1817 1818 27 1407 \
    > gpurun_out/r03p_probe.txt 2>&1
rc=$?
cat gpurun_out/r03p_probe.txt | grep -v amdgpu.ids
exit $rc
