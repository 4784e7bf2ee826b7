#!/bin/bash
# A/B of two in-tree builds of libvampomi on the operator at one shape, alternating:
#   bash tools/ab_lib.sh <alt .so> <N> <M> <plan> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
alt=$1 N=$2 M=$3 plan=$4 rounds=${5:-2}
for r in $(seq "$rounds"); do
    for lib in default "$alt"; do
        if [ "$lib" = default ]; then env_lib=(); else env_lib=(VAMPOMI_LIB="$lib"); fi
        echo "== $lib round $r"
        env "${env_lib[@]}" OP_PLANS="$plan" timeout -k 10 200 python tools/kbench.py "$N" "$M" 5 op \
            > gpurun_out/ab.log 2>&1
        rc=$?
        grep "^op " gpurun_out/ab.log
        if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.log; exit $rc; fi
    done
done
