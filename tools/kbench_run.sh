set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { timeout -k 10 300 python tools/kbench.py $1 $2 $3 ax > gpurun_out/kbn.log 2>&1 || { cat gpurun_out/kbn.log; exit 1; }
  echo "N=$1 Mt=$2: $(grep -E '^ax 0 ' gpurun_out/kbn.log | cut -c6-)"; }
run 100000 20000 8; run 50000 125000 4; run 200000 31250 4; run 25000 250000 4; run 100000 62500 4
