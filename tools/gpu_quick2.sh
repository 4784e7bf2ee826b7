set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_options.py -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -5 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c2.log
exit $rc
