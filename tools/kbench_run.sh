set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/quick_gpu.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_tr -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-timing > gpurun_out/prof_tr.log 2>&1 || { tail -20 gpurun_out/prof_tr.log; exit 1; }
f=$(find gpurun_out/prof_tr -name '*kernel_trace.csv' | head -1); python tools/trace_gaps.py "$f" 0.3
