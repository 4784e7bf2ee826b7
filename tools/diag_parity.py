"""Diagnose GPU-vs-oracle divergence iteration by iteration (run on the GPU box)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import vampomi_amd as va
from _data import make_problem
from oracle import pyoracle as O
from conftest import relerr

N, Mt = int(sys.argv[1]) if len(sys.argv) > 1 else 1000, int(sys.argv[2]) if len(sys.argv) > 2 else 2000
its = int(sys.argv[3]) if len(sys.argv) > 3 else 8
X, y, beta = make_problem(N, Mt)
for mi in (1, 2, its):
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=mi, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        d.load_meth(X); d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(max_iter=mi, stop_criteria_thr=0.0), true_signal=beta)
        v.infere(keep_hist=True)
        s = v.summary()
        print(f"--- max_iter={mi}: L gpu {v.r.L_final} orc {len(ref['probs_final'])}")
        print("probs rel", relerr(np.array(v.r.probs_final[:v.r.L_final]), ref["probs_final"]),
              "vars rel", relerr(np.array(v.r.vars_final[:v.r.L_final]), ref["vars_final"]))
        for k in range(mi):
            pg, po = np.array(s["params"][k]), ref["params"][k]
            print(k + 1, "x1 %.2e r1 %.2e" % (relerr(v.x1_hist[k, :Mt], ref["x1_hist"][k]),
                                            relerr(v.r1_hist[k, :Mt], ref["r1_hist"][k])),
                  "params rel", " ".join("%.1e" % (abs(a - b) / abs(b)) for a, b in zip(pg, po)),
                  "cg", s["cg_iters"][k], ref["cg_iters"][k], s["ons_iters"][k], ref["ons_iters"][k])

print("=== variants (max_iter 3)")
for name, kw in [("no-EM", dict(learn_prior_delay=100)), ("no-EM rho1", dict(learn_prior_delay=100, rho=1.0)),
                 ("EM rho1", dict(rho=1.0)), ("no-EM seq", dict(learn_prior_delay=100))]:
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=3, stop_criteria_thr=0.0, **kw)
    with va.Data(N, Mt) as d:
        d.load_meth(X); d.set_phen(y, standardize=False)
        opts = va.VampOptions(max_iter=3, stop_criteria_thr=0.0, batch_rhs=0 if "seq" in name else 1, **kw)
        v = va.Vamp(d, opts, true_signal=beta)
        v.infere(keep_hist=True)
        s = v.summary()
        for k in range(3):
            print(name, k + 1, "x1 %.2e r1 %.2e" % (relerr(v.x1_hist[k, :Mt], ref["x1_hist"][k]),
                                                  relerr(v.r1_hist[k, :Mt], ref["r1_hist"][k])),
                  "params", " ".join("%.1e" % (abs(a - b) / abs(b)) for a, b in zip(s["params"][k], ref["params"][k])))
