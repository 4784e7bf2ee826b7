#!/bin/bash
# The C2 operator with one component removed at COMPILE time (TM_ABL builds:
# make -C vampomi_amd/csrc EXTRA_FLAGS=-DTM_ABL=<bits> OBJDIR=../../build_abl<bits>/obj LIBDIR=... BINDIR=...),
# against the production library, alternating, each process with its own
# same-process read stream of the matrix:
#   bash tools/op_ablation_libs.sh [rounds]      (GPU box; output gpurun_out/ablation_libs.jsonl)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
out=gpurun_out/ablation_libs.jsonl
: > "$out"
for r in $(seq "${1:-3}"); do
    for lib in production build_abl8 build_abl2048 build_abl4096 build_abl6152; do
        if [ "$lib" = production ]; then env_lib=(); else env_lib=(VAMPOMI_LIB="$PWD/$lib/lib/libvampomi.so"); fi
        env "${env_lib[@]}" OP_ABL_ONE=1 timeout -k 10 120 python tools/op_ablation.py 10000 50000 40 >> "$out" || exit 1
        tail -n 1 "$out"
    done
done
