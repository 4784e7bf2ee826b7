#!/bin/bash
# C2 operator ablations (TM_DBG build in build_dbg/, tools/kbench.py op,
# default plan): which part of a step costs what.  VAMPOMI_OP_DBG bits
# (atax_team.hip): 1 no granule wait, 2 no publish (with 1), 4 no streaming
# butterfly, 8 no A d accumulation, 64 count slow polls, 256 no T-member sum.
#   gpurun -- bash tools/r03_ablate.sh [N Mt]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
N=${1:-10000}
MT=${2:-50000}
for dbg in ${DBGS:-0 64 256 1 3 4 8 12 0}; do
  VAMPOMI_LIB=$PWD/build_dbg/lib/libvampomi.so VAMPOMI_OP_DBG=$dbg OP_PLANS=-1 timeout -k 10 120 \
    python -u tools/kbench.py $N $MT 20 op > gpurun_out/r03a_dbg$dbg.txt 2>&1 || { echo "dbg $dbg failed"; tail -5 gpurun_out/r03a_dbg$dbg.txt; exit 1; }
  echo "dbg $dbg: $(grep '^op ' gpurun_out/r03a_dbg$dbg.txt | cut -c1-200) $(grep 'slow polls' gpurun_out/r03a_dbg$dbg.txt | tail -1)"
done
