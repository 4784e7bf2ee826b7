set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py 10000 50000 20 ax > gpurun_out/kbench_ax_c2.log 2>&1 || exit $?
grep -E "^ax " gpurun_out/kbench_ax_c2.log
timeout -k 10 300 python tools/kbench.py 50000 50000 6 ax > gpurun_out/kbench_ax_c4.log 2>&1 || exit $?
grep -E "^ax " gpurun_out/kbench_ax_c4.log
