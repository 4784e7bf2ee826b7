set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/kbench.py 10000 50000 20 ax,atx > gpurun_out/kbench_fma.log 2>&1; rc=$?
grep -E "^(ax|atx) " gpurun_out/kbench_fma.log; exit $rc
