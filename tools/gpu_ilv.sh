#!/bin/bash
# Team operator: contiguous marker ranges per team (cfg 6) against
# interleaved team columns (cfg 7: team t takes columns t, t + nteams, ...)
# at the large shapes, where the 8-16 teams' contiguous ranges lie far apart.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
OP_PLANS=326,327,328,326,327 timeout -k 10 300 python tools/kbench.py 100000 62500 10 op > gpurun_out/ilv_c3.txt 2>&1 || exit $?
cat gpurun_out/ilv_c3.txt
OP_PLANS=166,167,166,167 timeout -k 10 300 python tools/kbench.py 50000 200000 6 op > gpurun_out/ilv_c4full.txt 2>&1 || exit $?
cat gpurun_out/ilv_c4full.txt
OP_PLANS=326,327,328,326,327 timeout -k 10 400 python tools/kbench.py 100000 300000 4 ax,op > gpurun_out/ilv_c3big.txt 2>&1 || exit $?
cat gpurun_out/ilv_c3big.txt
