set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -2 gpurun_out/pt.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1; grep '^{' gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
