set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_corners.py tests/test_gpu_sharded.py -x -q > gpurun_out/kb_tests.log 2>&1 || { tail -30 gpurun_out/kb_tests.log; exit 1; }
tail -1 gpurun_out/kb_tests.log
run() { VAMPOMI_AX_BANDSEG=$4 timeout -k 10 300 python tools/kbench.py $1 $2 $3 ax > gpurun_out/kbn.log 2>&1 || { cat gpurun_out/kbn.log; exit 1; }
  echo "N=$1 Mt=$2 bandseg=$4: $(grep -E '^ax 0 ' gpurun_out/kbn.log | cut -c6-)"; }
for s in 32 64 128 256 0; do run 10000 50000 20 $s; done
for s in 32 64 128 256 0; do run 50000 50000 6 $s; done
for s in 32 64 128 256 0; do run 100000 62500 4 $s; done
