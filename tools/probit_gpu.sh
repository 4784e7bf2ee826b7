set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_probit.py -q -rf > gpurun_out/probit_tests.log 2>&1; rc=$?
echo "probit tests rc=$rc"; tail -30 gpurun_out/probit_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?
echo "bench c4 rc=$rc"; tail -3 gpurun_out/bench_c4.log
