"""ctypes wrapper of the CPU restatement (oracle/vamp_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / the timed CPU baseline,
never as the product path.  PARITY UNPINNED: see vamp_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Callable, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libvamp_oracle.so")
MAX_L = 64

ALLREDUCE_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int64, C.c_void_p)


class Problem(C.Structure):
    _fields_ = [("N", C.c_int64), ("Mt", C.c_int64), ("M", C.c_int64), ("S", C.c_int64), ("ld", C.c_int64),
                ("rank", C.c_int), ("nranks", C.c_int),
                ("X", C.c_void_p), ("mave", C.c_void_p), ("msig", C.c_void_p), ("y", C.c_void_p),
                ("true_signal", C.c_void_p), ("x1hat_init", C.c_void_p),
                ("allreduce", ALLREDUCE_FN), ("user", C.c_void_p)]


class Params(C.Structure):
    _fields_ = [("gam1", C.c_double), ("h2", C.c_double), ("max_iter", C.c_int), ("CG_max_iter", C.c_int),
                ("CG_err_tol", C.c_double), ("EM_max_iter", C.c_int), ("EM_err_thr", C.c_double),
                ("rho", C.c_double), ("learn_vars", C.c_int), ("learn_prior_delay", C.c_int),
                ("stop_criteria_thr", C.c_double), ("merge_vars_thr", C.c_double), ("L", C.c_int),
                ("vars", C.c_double * MAX_L), ("probs", C.c_double * MAX_L), ("seed", C.c_uint64),
                ("out_dir", C.c_char_p), ("out_name", C.c_char_p), ("verbosity", C.c_int)]


class Result(C.Structure):
    _fields_ = [("iterations_run", C.c_int), ("cg_iters", C.c_void_p), ("ons_iters", C.c_void_p),
                ("L_hist", C.c_void_p), ("params", C.c_void_p), ("metrics", C.c_void_p),
                ("x1_hist", C.c_void_p), ("r1_hist", C.c_void_p), ("x1_final", C.c_void_p),
                ("probs_final", C.c_void_p), ("vars_final", C.c_void_p), ("L_final", C.c_int),
                ("a_passes", C.c_int64), ("prior_hist", C.c_void_p), ("it_wall", C.c_void_p),
                ("wall_start", C.c_double)]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C oracle`")
        lib = C.CDLL(LIB_PATH)
        d, p, i64 = C.c_double, C.c_void_p, C.c_int64
        lib.orc_splitmix64.restype = C.c_uint64
        lib.orc_splitmix64.argtypes = [C.c_uint64]
        lib.orc_bern_bit.restype = C.c_int
        lib.orc_bern_bit.argtypes = [C.c_uint64, C.c_int, i64]
        lib.orc_gauss_dyadic.restype = d
        lib.orc_gauss_dyadic.argtypes = [C.c_uint64, i64, i64]
        lib.orc_meth_dyadic.restype = d
        lib.orc_meth_dyadic.argtypes = [C.c_uint64, i64, i64]
        lib.orc_generate_markers.argtypes = [C.c_uint64, C.c_int, i64, i64, i64, i64, p]
        lib.orc_divide_work.argtypes = [i64, C.c_int, C.c_int, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
        lib.orc_read_phen.restype = i64
        lib.orc_read_phen.argtypes = [C.c_char_p, C.c_int, p, i64, C.POINTER(d), C.POINTER(d)]
        lib.orc_standardize_phen.argtypes = [p, i64]
        lib.orc_marker_stats.argtypes = [p, i64, i64, i64, i64, d, p, p]
        lib.orc_ax_local.argtypes = [p, i64, i64, i64, p, p, p, p]
        lib.orc_ax.argtypes = [p, i64, i64, i64, p, p, p, p, ALLREDUCE_FN, p]
        lib.orc_atx.argtypes = [p, i64, i64, i64, p, p, p, p]
        lib.orc_set_atx_block.argtypes = [C.c_int]
        lib.orc_set_assoc.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64]
        lib.orc_assoc_dot.restype = d
        lib.orc_assoc_dot.argtypes = [p, p, i64, C.c_int]
        lib.orc_dev_dp.restype = d
        lib.orc_dev_dp.argtypes = [p, p, i64, C.c_int, C.c_int]
        lib.orc_g1.restype = d
        lib.orc_g1.argtypes = [d, d, p, p, C.c_int]
        lib.orc_g1d.restype = d
        lib.orc_g1d.argtypes = [d, d, p, p, C.c_int]
        lib.orc_dot.restype = d
        lib.orc_dot.argtypes = [p, p, i64]
        lib.orc_vamp_infere_linear.restype = C.c_int
        lib.orc_vamp_infere_linear.argtypes = [C.POINTER(Problem), C.POINTER(Params), C.POINTER(Result)]
        lib.orc_store_vec.argtypes = [C.c_char_p, p, i64, i64]
        lib.orc_vamp_infere_probit.restype = C.c_int
        lib.orc_vamp_infere_probit.argtypes = [C.POINTER(Problem), C.POINTER(Params), C.POINTER(Result)]
        lib.orc_probit_p1.restype = d
        lib.orc_probit_p1.argtypes = [C.c_uint64, i64]
        lib.orc_erfcx.restype = d
        lib.orc_erfcx.argtypes = [d]
        for f in (lib.orc_g1_bin, lib.orc_g1d_bin):
            f.restype = d
            f.argtypes = [d, d, d]
        lib.orc_t_sf.restype = d
        lib.orc_t_sf.argtypes = [d, d]
        lib.orc_lnbeta_half.restype = d
        lib.orc_lnbeta_half.argtypes = [d]
        lib.orc_reg1d_pval.restype = d
        lib.orc_reg1d_pval.argtypes = [d, d, d, d, d, C.c_int]
        lib.orc_assoc_loo.argtypes = [C.POINTER(Problem), p, p, p]
        lib.orc_assoc_se.argtypes = [p, i64, d, i64, p]
        lib.orc_test_metrics.argtypes = [C.POINTER(Problem), p, p]
        lib.orc_update_prior.restype = C.c_int
        lib.orc_update_prior.argtypes = [C.POINTER(Problem), p, d, C.POINTER(Params), C.POINTER(C.c_int), p, p]
        _lib = lib
    return _lib


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def divide_work(Mt: int, nranks: int, rank: int):
    M, S, Mm = C.c_int64(), C.c_int64(), C.c_int64()
    load().orc_divide_work(Mt, nranks, rank, C.byref(M), C.byref(S), C.byref(Mm))
    return M.value, S.value, Mm.value


def generate_markers(seed: int, kind: int, N: int, S: int, M: int) -> np.ndarray:
    """(M, N) marker-major shard of the synthetic design (global markers S..S+M)."""
    X = np.empty((M, N))
    load().orc_generate_markers(seed, kind, N, N, S, M, _p(X))
    return X


def bern_bits(seed: int, it: int, S: int, M: int) -> np.ndarray:
    lib = load()
    return np.array([lib.orc_bern_bit(seed, it, S + i) for i in range(M)], dtype=np.int64)


def marker_stats(X: np.ndarray, alpha_scale: float = 1.0):
    M, N = X.shape
    mave, msig = np.empty(M), np.empty(M)
    load().orc_marker_stats(_p(X), N, N, M, N, alpha_scale, _p(mave), _p(msig))
    return mave, msig


def ax(X, mave, msig, x, allreduce: Optional[Callable] = None) -> np.ndarray:
    M, N = X.shape
    out = np.empty(N)
    if allreduce is None:
        load().orc_ax(_p(X), N, N, M, _p(mave), _p(msig), _p(np.ascontiguousarray(x, dtype=np.float64)), _p(out),
                      ALLREDUCE_FN(), None)
    else:
        cb = _make_allreduce(allreduce)
        load().orc_ax(_p(X), N, N, M, _p(mave), _p(msig), _p(np.ascontiguousarray(x, dtype=np.float64)), _p(out),
                      cb, None)
    return out


def atx(X, mave, msig, u) -> np.ndarray:
    M, N = X.shape
    out = np.empty(M)
    load().orc_atx(_p(X), N, N, M, _p(mave), _p(msig), _p(np.ascontiguousarray(u, dtype=np.float64)), _p(out))
    return out


def set_omp_threads(n: int) -> None:
    """OpenMP team size of the oracle's parallel loops started from the
    calling thread (omp_set_num_threads sets the calling thread's ICV)."""
    global _gomp
    if _gomp is None:
        load()
        _gomp = C.CDLL("libgomp.so.1")
        _gomp.omp_set_num_threads.argtypes = [C.c_int]
    _gomp.omp_set_num_threads(int(n))


_gomp = None


def set_atx_block(B: int) -> None:
    """Sensitivity mode: A^T.u sums samples in blocks of B rows (0 = off)."""
    load().orc_set_atx_block(int(B))


ASSOC_DEFAULT, ASSOC_DEVICE, ASSOC_REFRUN = 0, 1, 2


def set_assoc(mode: int = ASSOC_DEFAULT, a: int = 0, b: int = 0, seed: int = 0) -> None:
    """Association mode of the scalar sums (vamp_oracle.c; single-rank runs):
    ASSOC_DEVICE with a = team size T, b = workgroups of the engine's operator
    plan; ASSOC_REFRUN with a = OpenMP threads of one reference rank and the
    seed of its threads' arrival order; ASSOC_DEFAULT the restatement."""
    load().orc_set_assoc(int(mode), int(a), int(b), int(seed) & (2**64 - 1))


def g1(y: float, gam1: float, probs, vars_scaled) -> float:
    pr = np.ascontiguousarray(probs, dtype=np.float64)
    va = np.ascontiguousarray(vars_scaled, dtype=np.float64)
    return load().orc_g1(y, gam1, _p(pr), _p(va), len(pr))


def g1d(y: float, gam1: float, probs, vars_scaled) -> float:
    pr = np.ascontiguousarray(probs, dtype=np.float64)
    va = np.ascontiguousarray(vars_scaled, dtype=np.float64)
    return load().orc_g1d(y, gam1, _p(pr), _p(va), len(pr))


def erfcx(x: float) -> float:
    return load().orc_erfcx(x)


def g1_bin(p: float, tau1: float, y: float) -> float:
    return load().orc_g1_bin(p, tau1, y)


def g1d_bin(p: float, tau1: float, y: float) -> float:
    return load().orc_g1d_bin(p, tau1, y)


def probit_p1(seed: int, N: int) -> np.ndarray:
    lib = load()
    return np.array([lib.orc_probit_p1(seed, i) for i in range(N)])


def t_sf(t: float, df: float) -> float:
    return load().orc_t_sf(t, df)


def reg1d_pval(sumx, sumsqx, sumxy, sumy, sumsqy, n: int) -> float:
    return load().orc_reg1d_pval(sumx, sumsqx, sumxy, sumy, sumsqy, n)


def assoc_loo(X: np.ndarray, y: np.ndarray, est: np.ndarray, Mt: Optional[int] = None, S: int = 0, rank: int = 0,
              nranks: int = 1, allreduce: Optional[Callable] = None, alpha_scale: float = 1.0):
    """--pval-method loo on one shard X (M, N): returns (pvals, stats (M, 5))."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    M, N = X.shape
    y = np.ascontiguousarray(y, dtype=np.float64)
    est = np.ascontiguousarray(est, dtype=np.float64)
    mave, msig = marker_stats(X, alpha_scale)
    cb = _make_allreduce(allreduce) if allreduce is not None else ALLREDUCE_FN()
    pb = Problem(N=N, Mt=Mt or M, M=M, S=S, ld=N, rank=rank, nranks=nranks, X=_p(X), mave=_p(mave), msig=_p(msig),
                 y=_p(y), true_signal=None, x1hat_init=None, allreduce=cb, user=None)
    pv = np.zeros(max(M, 1))
    st = np.zeros((max(M, 1), 5))
    lib.orc_assoc_loo(C.byref(pb), _p(est), _p(pv), _p(st))
    return pv[:M], st[:M]


def test_metrics(X: np.ndarray, y: np.ndarray, est: np.ndarray, alpha_scale: float = 1.0):
    """--run-mode test row for one estimate (one shard, X (M, N_test)): (R2 test, corr^2)."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    M, N = X.shape
    y = np.ascontiguousarray(y, dtype=np.float64)
    est = np.ascontiguousarray(est, dtype=np.float64)
    mave, msig = marker_stats(X, alpha_scale)
    pb = Problem(N=N, Mt=M, M=M, S=0, ld=N, rank=0, nranks=1, X=_p(X), mave=_p(mave), msig=_p(msig), y=_p(y),
                 true_signal=None, x1hat_init=None, allreduce=ALLREDUCE_FN(), user=None)
    out = np.zeros(2)
    lib.orc_test_metrics(C.byref(pb), _p(est), _p(out))
    return float(out[0]), float(out[1])


test_metrics.__test__ = False  # not a pytest test


def update_prior(r1: np.ndarray, gam1: float, probs, vars_scaled, N: int, Mt: Optional[int] = None,
                 EM_max_iter=1, EM_err_thr=1e-2, learn_vars=1, merge_vars_thr=0.5):
    """updatePrior (src/vamp.cpp:531-643) on one shard's r1: returns (probs, vars)."""
    lib = load()
    r1 = np.ascontiguousarray(r1, dtype=np.float64)
    M = len(r1)
    pb = Problem(N=N, Mt=Mt or M, M=M, S=0, ld=N, rank=0, nranks=1, X=None, mave=None, msig=None, y=None,
                 true_signal=None, x1hat_init=None, allreduce=ALLREDUCE_FN(), user=None)
    pr = Params(EM_max_iter=EM_max_iter, EM_err_thr=EM_err_thr, learn_vars=learn_vars, merge_vars_thr=merge_vars_thr)
    L = C.c_int(len(probs))
    pp, vv = np.zeros(MAX_L), np.zeros(MAX_L)
    pp[: L.value] = probs
    vv[: L.value] = vars_scaled
    if lib.orc_update_prior(C.byref(pb), _p(r1), gam1, C.byref(pr), C.byref(L), _p(pp), _p(vv)) != 0:
        raise ValueError("bad mixture")
    return pp[: L.value].copy(), vv[: L.value].copy()


def assoc_se(r1: np.ndarray, gam1: float, N: int) -> np.ndarray:
    r1 = np.ascontiguousarray(r1, dtype=np.float64)
    out = np.zeros(max(len(r1), 1))
    load().orc_assoc_se(_p(r1), len(r1), gam1, N, _p(out))
    return out[:len(r1)]


def read_phen(path: str, N: int, standardize: bool = True) -> np.ndarray:
    y = np.zeros(N)
    n = load().orc_read_phen(path.encode(), 1 if standardize else 0, _p(y), N, None, None)
    if n < 0:
        raise IOError(f"read_phen({path}) -> {n}")
    return y[:n]


def standardize_phen(y: np.ndarray) -> np.ndarray:
    y = np.array(y, dtype=np.float64)
    load().orc_standardize_phen(_p(y), len(y))
    return y


def _make_allreduce(fn: Callable[[np.ndarray], None]):
    def cb(buf, n, user):
        a = np.ctypeslib.as_array(buf, shape=(n,))
        fn(a)
    return ALLREDUCE_FN(cb)


DEFAULT_VARS = (0, 1e-06, 6e-06, 3e-05, 2e-04, 1e-03, 6e-03, 3e-02, 2e-01, 1e+00)
DEFAULT_PROBS = (9.9e-01, 5e-03, 2.5e-03, 1.25e-03, 6.25e-04, 3.125e-04, 1.5625e-04, 7.8125e-05, 3.90625e-05,
                 3.90625e-05)


def vamp_infere(X: np.ndarray, y: np.ndarray, Mt: int, S: int = 0, rank: int = 0, nranks: int = 1, *,
                true_signal=None, x1hat_init=None, allreduce: Optional[Callable] = None,
                gam1=1e-6, h2=0.5, max_iter=50, CG_max_iter=500, CG_err_tol=1e-5, EM_max_iter=1, EM_err_thr=1e-2,
                rho=0.5, learn_vars=1, learn_prior_delay=1, stop_criteria_thr=0.01, merge_vars_thr=0.5,
                vars: Sequence[float] = DEFAULT_VARS, probs: Sequence[float] = DEFAULT_PROBS,
                seed=0x5EED5EED, out_dir="", out_name="", verbosity=0, alpha_scale=1.0, keep_hist=True,
                model="linear") -> dict:
    """Run the restated infere_linear (model="linear") or infere_bin_class
    (model="bin_class", y = raw 0/1 phenotype) on one shard X (M, N)."""
    probit = model == "bin_class"
    if model not in ("linear", "bin_class"):
        raise ValueError(model)
    npar, nmet = (8, 12) if probit else (5, 6)
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    M, N = X.shape
    y = np.ascontiguousarray(y, dtype=np.float64)
    mave, msig = marker_stats(X, alpha_scale)
    ts = None if true_signal is None else np.ascontiguousarray(true_signal, dtype=np.float64)
    xi = None if x1hat_init is None else np.ascontiguousarray(x1hat_init, dtype=np.float64)
    cb = _make_allreduce(allreduce) if allreduce is not None else ALLREDUCE_FN()
    pb = Problem(N=N, Mt=Mt, M=M, S=S, ld=N, rank=rank, nranks=nranks, X=_p(X), mave=_p(mave), msig=_p(msig),
                 y=_p(y), true_signal=_p(ts), x1hat_init=_p(xi), allreduce=cb, user=None)
    pr = Params(gam1=gam1, h2=h2, max_iter=max_iter, CG_max_iter=CG_max_iter, CG_err_tol=CG_err_tol,
                EM_max_iter=EM_max_iter, EM_err_thr=EM_err_thr, rho=rho, learn_vars=learn_vars,
                learn_prior_delay=learn_prior_delay, stop_criteria_thr=stop_criteria_thr,
                merge_vars_thr=merge_vars_thr, L=len(vars), seed=seed, out_dir=out_dir.encode(),
                out_name=out_name.encode(), verbosity=verbosity)
    for j, (v, q) in enumerate(zip(vars, probs)):
        pr.vars[j] = v
        pr.probs[j] = q
    cg = np.zeros(max_iter, dtype=np.int32)
    ons = np.zeros(max_iter, dtype=np.int32)
    Lh = np.zeros(max_iter, dtype=np.int32)
    params = np.zeros((max_iter, npar))
    metrics = np.zeros((max_iter, nmet))
    prior = np.zeros((max_iter, 1 + 2 * MAX_L)) if probit else None
    x1h = np.zeros((max_iter, max(M, 1))) if keep_hist else None
    r1h = np.zeros((max_iter, max(M, 1))) if keep_hist else None
    x1f = np.zeros(max(M, 1))
    pf, vf = np.zeros(MAX_L), np.zeros(MAX_L)
    wall = np.zeros(max_iter)
    res = Result(cg_iters=_p(cg), ons_iters=_p(ons), L_hist=_p(Lh), params=_p(params), metrics=_p(metrics),
                 x1_hist=_p(x1h), r1_hist=_p(r1h), x1_final=_p(x1f), probs_final=_p(pf), vars_final=_p(vf),
                 prior_hist=_p(prior), it_wall=_p(wall))
    fn = lib.orc_vamp_infere_probit if probit else lib.orc_vamp_infere_linear
    rc = fn(C.byref(pb), C.byref(pr), C.byref(res))
    if rc != 0:
        raise RuntimeError(f"{fn.__name__} -> {rc}")
    n = res.iterations_run
    out = {"iterations": n, "cg_iters": cg[:n].copy(), "ons_iters": ons[:n].copy(), "L": Lh[:n].copy(),
           "params": params[:n].copy(), "metrics": metrics[:n].copy(), "x1_final": x1f[:M].copy(),
           "probs_final": pf[:res.L_final].copy(), "vars_final": vf[:res.L_final].copy(), "a_passes": res.a_passes,
           "mave": mave, "msig": msig,
           # seconds from the start of iteration 1 to the end of each iteration (timing only)
           "it_end_s": wall[:n] - res.wall_start}
    if probit:
        out["prior"] = prior[:n].copy()
    if keep_hist:
        out["x1_hist"] = x1h[:n, :M].copy()
        out["r1_hist"] = r1h[:n, :M].copy()
    return out
