set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config c3big --steps 4 --warmup 1 > gpurun_out/bench_c3big.log 2>&1 || { tail -20 gpurun_out/bench_c3big.log; exit 1; }
tail -1 gpurun_out/bench_c3big.log
