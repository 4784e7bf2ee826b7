"""Diagnostic: every operator plan of one shape, one launch at a time (K = 1,
then 2), printing the plan before each launch, checked against numpy.
    python tools/op_plan_probe.py N Mt [variants...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import vampomi_amd as va  # noqa: E402
from oracle import pyoracle as O  # noqa: E402
from test_gpu_operator import _ref  # noqa: E402

N, Mt = int(sys.argv[1]), int(sys.argv[2])
vs = [int(v) for v in sys.argv[3:]]
X = O.generate_markers(11, 0, N, 0, Mt)
mave, msig = O.marker_stats(X)
d = va.Data(N, Mt)
d.load_meth(X)
rng = np.random.default_rng(N)
for v in vs:
    try:
        d.set_variant(3, v)
    except va.VampomiError as e:
        print(v, "no plan", e, flush=True)
        continue
    for K in (1, 2):
        ar, p = rng.normal(size=(K, N)), rng.normal(size=(K, Mt))
        print(v, d.kernel_name(3, K), "K", K, "...", end=" ", flush=True)
        try:
            gd, gad, gdp = d.op_apply(ar, p, 1.7, 0.9, 0.35)
        except va.VampomiError as e:
            print("ERROR", e, flush=True)
            sys.exit(1)
        rd, rad, rdp = _ref(X, mave, msig, ar, None, p, None, None, 1.7, 0.9, 0.35)
        e1 = np.linalg.norm(gd - rd) / np.linalg.norm(rd)
        e2 = np.linalg.norm(gad - rad) / np.linalg.norm(rad)
        print("d %.1e  Ad %.1e" % (e1, e2), flush=True)
d.close()
