#!/bin/bash
# the whole -m gpu suite, the C2 bench with --write, and the CLI with / without files
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03v}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --write --no-cpu-baseline \
    > gpurun_out/${tag}_bench_c2.json 2> gpurun_out/${tag}_bench_c2.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench_c2.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], 'with_writes', d['with_writes']['value'], d['with_writes']['rate_vs_no_write'])"
timeout -k 10 600 python -u tools/cli_write_ab.py /tmp 3 > gpurun_out/${tag}_cli_write.txt 2>&1 || { echo cli failed; tail gpurun_out/${tag}_cli_write.txt; exit 1; }
tail -1 gpurun_out/${tag}_cli_write.txt
