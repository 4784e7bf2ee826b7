"""Bitwise comparison of two libvampomi builds (a refactor that must not move
a bit: same kernels' summation orders).  Each run is its own process (the
library is chosen at load by VAMPOMI_LIB):

    python tools/lib_bitwise.py run OUT.npz [N Mt iters model]   # one build
    python tools/lib_bitwise.py cmp A.npz B.npz                   # exit 1 on any difference

A run saves x1_hat/r1 of every iteration, the parameters, metrics and every
integer count of a VAMP run on the device-generated problem (the bench's
generator and seeds)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def run(out, N=10000, Mt=20000, iters=12, model="linear"):
    import torch  # noqa: F401  (one HIP runtime per process)

    import vampomi_amd as va

    d = va.Data(N, Mt)
    d.generate(20250711, va.GEN_GAUSS)
    beta = (d.simulate_phen_binary if model == "bin_class" else d.simulate_phen)(20250712, lam=0.1, h2=0.8)
    v = va.Vamp(d, va.VampOptions(max_iter=iters, stop_criteria_thr=0.0, model=model), true_signal=beta)
    v.infere(keep_hist=True)
    s = v.summary()
    np.savez(out, x1=v.x1_hist, r1=v.r1_hist, params=np.array(s["params"]), metrics=np.array(s["metrics"]),
             cg=np.array(s["cg_iters"]), ons=np.array(s["ons_iters"]), L=np.array(s["L"]),
             lib=np.array(os.environ.get("VAMPOMI_LIB", "default")))
    d.close()
    print("saved", out, "cg", s["cg_iters"], "ons", s["ons_iters"])


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = []
    for k in ("x1", "r1", "params", "metrics", "cg", "ons", "L"):
        same = np.array_equal(A[k], B[k], equal_nan=True) if A[k].dtype.kind == "f" else np.array_equal(A[k], B[k])
        if not same:
            bad.append(k)
    print("bitwise equal" if not bad else "DIFFER: %s" % bad, "(%s vs %s)" % (A["lib"], B["lib"]))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        args = [int(x) for x in sys.argv[3:6]] + sys.argv[6:7]
        run(sys.argv[2], *args)
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
