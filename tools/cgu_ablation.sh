#!/bin/bash
# cg_update with one part removed at COMPILE time (CGU_ABL builds, results wrong:
# make -C vampomi_amd/csrc EXTRA_FLAGS=-DCGU_ABL=<bits> OBJDIR=../../build_cgu<bits>/obj LIBDIR=... BINDIR=...;
# 1 = no slot sums / N-side updates, 2 = no M-side loads / stores, 3 = both: the
# state, the ticket and the decision alone), against the production library:
# tools/cgu_bench.hip (build_cgu/cgu_bench) times back-to-back launches alone at
# the C2 and C4 shapes, alternating the libraries.
#   bash tools/cgu_ablation.sh <tag> [rounds]      (GPU box; output gpurun_out/<tag>/cgu.txt;
#   LIBS="<lib dir> ...": other libraries, e.g. a saved copy of the previous build)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
for r in $(seq "${2:-3}"); do
    for lib in ${LIBS:-vampomi_amd/lib build_cgu1/lib build_cgu2/lib build_cgu3/lib}; do
        for shape in "10000 50000 128" "50000 50000 16"; do
            line=$(LD_LIBRARY_PATH="$PWD/$lib" timeout -k 10 60 build_cgu/cgu_bench $shape 400) || {
                echo "failed: $lib $shape"; exit 1; }
            echo "$r $lib $line" | tee -a "$OUT/cgu.txt"
        done
    done
done
