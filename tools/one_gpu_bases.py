"""GPU check of bench.py's rank-0 1-GPU bases outside a job (no gloo): runs
one_gpu_bases for a 2-rank c2-weak line and prints what it returns."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

import bench  # noqa: E402
from vampomi_amd.workloads import workload  # noqa: E402


class R:
    world, rank, local = 2, 0, 0

    def barrier(self):
        pass


class Wd:
    def stage(self, s):
        print("stage:", s, flush=True)


args = bench.parse_args(["--gpus", "2", "--steps", "5", "--warmup", "2"])
t0 = time.time()
out = bench.one_gpu_bases(args, R(), Wd(), workload("auto", 2), True)
print(json.dumps(out), flush=True)
print("took", round(time.time() - t0, 1), "s")
