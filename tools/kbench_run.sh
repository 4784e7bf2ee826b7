set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { VAMPOMI_LOO_WPB=$4 timeout -k 10 300 python tools/kbench.py $1 $2 $3 loo > gpurun_out/kbn.log 2>&1 || { cat gpurun_out/kbn.log; exit 1; }
  echo "N=$1 Mt=$2 loo wpb=$4"; grep -E '^loo [0-3] ' gpurun_out/kbn.log | cut -c1-160; }
for w in 4 2 1; do run 100000 62500 4 $w; done
for w in 4 2; do run 10000 50000 20 $w; done
timeout -k 10 300 python tools/kbench.py 10000 50000 20 atx > gpurun_out/kbn.log 2>&1 && grep -E '^atx [0234] ' gpurun_out/kbn.log | cut -c1-120
