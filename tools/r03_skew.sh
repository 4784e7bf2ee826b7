#!/bin/bash
# operator workgroup skew (TM_TS build in vampomi_amd/lib_ts) at C2 and the C3 shard
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03s}
export VAMPOMI_LIB=$PWD/vampomi_amd/lib_ts/libvampomi.so VAMPOMI_OP_TS=1
timeout -k 10 120 python -u tools/op_skew.py 10000 50000 6 2 > gpurun_out/${tag}_skew_c2.txt 2>&1 || { echo c2 failed; tail -20 gpurun_out/${tag}_skew_c2.txt; exit 1; }
cat gpurun_out/${tag}_skew_c2.txt | cut -c1-400
timeout -k 10 120 python -u tools/op_skew.py 10000 50000 4 1 > gpurun_out/${tag}_skew_c2k1.txt 2>&1 || { echo c2k1 failed; exit 1; }
tail -2 gpurun_out/${tag}_skew_c2k1.txt | cut -c1-300
timeout -k 10 300 python -u tools/op_skew.py 100000 62500 4 2 > gpurun_out/${tag}_skew_c3.txt 2>&1 || { echo c3 failed; tail -20 gpurun_out/${tag}_skew_c3.txt; exit 1; }
cat gpurun_out/${tag}_skew_c3.txt | cut -c1-400
