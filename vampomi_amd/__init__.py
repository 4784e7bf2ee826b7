"""vampomi_amd — MI355X-native gVAMPomi VAMP engine (host-side mirror).

The compute lives in libvampomi.so (HIP kernels for gfx950 + RCCL, C ABI in
include/vampomi.h).  This module mirrors the reference's operator interface
so code written against it reads like the reference:

* :class:`Data` — the reference's ``class data`` (src/data.hpp:11-92):
  phenotype + marker-major fp64 shard, ``Ax`` / ``ATx`` / ``get_mave`` /
  ``get_msig`` / ``get_phen``;
* :class:`Vamp` — the reference's ``class vamp`` (src/vamp.hpp:7-151):
  ``infere`` runs ``infere_linear`` on the device, plus the step-wise API used
  by bench.py;
* :func:`divide_work` — src/utilities.cpp:207-239.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from ._lib import (CLI_PATH, GEN_GAUSS, GEN_METH, LIB_PATH, MAX_L, MEM_DEVICE, MEM_HOST, UNIQUE_ID_BYTES,
                   Params, Result, ShardDesc, Stats, VampomiError, check, load)

__all__ = ["Data", "Vamp", "VampOptions", "divide_work", "comm_unique_id", "VampomiError", "LIB_PATH", "CLI_PATH",
           "GEN_GAUSS", "GEN_METH", "load"]


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def divide_work(Mt: int, nranks: int, rank: int):
    """(M, S, Mm) of ``rank`` — src/utilities.cpp:207-239."""
    M, S, Mm = C.c_int64(), C.c_int64(), C.c_int64()
    load().vampomi_divide_work(Mt, nranks, rank, C.byref(M), C.byref(S), C.byref(Mm))
    return M.value, S.value, Mm.value


def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it, the caller broadcasts it)."""
    buf = (C.c_ubyte * UNIQUE_ID_BYTES)()
    check(load().vampomi_comm_unique_id(buf))
    return bytes(buf)


class Data:
    """Device-resident marker shard + phenotype (reference ``class data``).

    ``Data(N, Mt, rank, nranks)`` owns markers ``[S, S+M)`` of ``Mt``
    (divide_work).  Load the shard with :meth:`read_methylation_data` (file),
    :meth:`load_meth` (numpy, shape (M, N) marker-major) or :meth:`generate`
    (on-device synthetic); the phenotype with :meth:`read_phen` or
    :meth:`set_phen`.  Marker statistics are computed at load
    (compute_markers_statistics, src/data.cpp:233-283).
    """

    def __init__(self, N: int, Mt: int, rank: int = 0, nranks: int = 1, comm_id: Optional[bytes] = None,
                 device: int = -1, alpha_scale: float = 1.0):
        self._lib = load()
        self._idbuf = None
        d = ShardDesc(N=N, Mt=Mt, rank=rank, nranks=nranks, device=device, comm_id=None, alpha_scale=alpha_scale)
        if nranks > 1:
            if comm_id is None or len(comm_id) != UNIQUE_ID_BYTES:
                raise ValueError("nranks > 1 needs the 128-byte communicator id from rank 0")
            self._idbuf = (C.c_ubyte * UNIQUE_ID_BYTES).from_buffer_copy(comm_id)
            d.comm_id = C.cast(self._idbuf, C.c_void_p)
        h = C.c_void_p()
        check(self._lib.vampomi_open(C.byref(d), C.byref(h)))
        self.ctx = h
        self.N, self.Mt, self.rank, self.nranks = N, Mt, rank, nranks
        M, S, ld = C.c_int64(), C.c_int64(), C.c_int64()
        check(self._lib.vampomi_shard_info(self.ctx, C.byref(M), C.byref(S), C.byref(ld)))
        self.M, self.S, self.ld = M.value, S.value, ld.value

    # -- lifecycle --
    def close(self):
        if getattr(self, "ctx", None):
            self._lib.vampomi_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def sync(self):
        check(self._lib.vampomi_sync(self.ctx))

    def barrier(self):
        check(self._lib.vampomi_barrier(self.ctx))

    # -- ingest --
    def read_methylation_data(self, path: str):
        check(self._lib.vampomi_load_meth_file(self.ctx, path.encode()))

    def load_meth(self, X: np.ndarray):
        """X: (M, N) float64, this shard's markers (marker-major)."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.shape != (self.M, self.N):
            raise ValueError(f"expected shard shape {(self.M, self.N)}, got {X.shape}")
        check(self._lib.vampomi_load_meth_host(self.ctx, _dp(X), self.N))

    def generate(self, seed: int, kind: int = GEN_GAUSS):
        check(self._lib.vampomi_generate_meth(self.ctx, seed, kind))

    def read_phen(self, path: str, standardize: bool = True):
        check(self._lib.vampomi_read_phen(self.ctx, path.encode(), 1 if standardize else 0))

    def set_phen(self, y: np.ndarray, standardize: bool = True):
        y = np.ascontiguousarray(y, dtype=np.float64)
        if y.shape != (self.N,):
            raise ValueError("phenotype must have N entries")
        check(self._lib.vampomi_set_phen(self.ctx, _dp(y), 1 if standardize else 0))

    def simulate_phen_binary(self, seed: int, lam: float = 0.1, h2: float = 0.8) -> np.ndarray:
        """Liability of simulate_phen thresholded at 0, stored raw (bin_class); returns beta."""
        beta = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_simulate_phen_binary(self.ctx, seed, lam, h2, _dp(beta)))
        return beta[: self.M]

    def simulate_phen(self, seed: int, lam: float = 0.1, h2: float = 0.8) -> np.ndarray:
        beta = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_simulate_phen(self.ctx, seed, lam, h2, _dp(beta)))
        return beta[: self.M]

    # -- accessors (src/data.hpp:48-66) --
    def get_phen(self) -> np.ndarray:
        y = np.zeros(self.N)
        check(self._lib.vampomi_get_phen(self.ctx, _dp(y)))
        return y

    def get_mave(self) -> np.ndarray:
        a = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_get_marker_stats(self.ctx, _dp(a), None))
        return a[: self.M]

    def get_msig(self) -> np.ndarray:
        a = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_get_marker_stats(self.ctx, None, _dp(a)))
        return a[: self.M]

    def get_meth_data(self, i0: int = 0, count: Optional[int] = None) -> np.ndarray:
        """Local markers [i0, i0+count) as a (count, N) array (src/data.hpp:53)."""
        count = self.M - i0 if count is None else count
        out = np.zeros((max(count, 1), self.N))
        check(self._lib.vampomi_read_markers(self.ctx, i0, count, _dp(out)))
        return out[:count]

    # -- operators (src/data.cpp:294-373) --
    def Ax(self, x: np.ndarray) -> np.ndarray:
        """COLLECTIVE: (sum over ranks of (X - mave) * msig * x) / sqrt(N)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros(self.N)
        check(self._lib.vampomi_ax(self.ctx, _dp(x), _dp(out), MEM_HOST))
        return out

    def ATx(self, u: np.ndarray) -> np.ndarray:
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_atx(self.ctx, _dp(u), _dp(out), MEM_HOST))
        return out[: self.M]

    def lmmse_mult(self, v: np.ndarray, tau: float, gam2: float) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_lmmse_mult(self.ctx, _dp(v), tau, gam2, _dp(out), MEM_HOST))
        return out[: self.M]

    def pcg(self, v: np.ndarray, tau: float, gam2: float, mu0: Optional[np.ndarray] = None, onsager: bool = False,
            max_iter: int = 500, tol: float = 1e-5):
        v = np.ascontiguousarray(v, dtype=np.float64)
        mu = np.zeros(max(self.M, 1))
        it = C.c_int()
        m0 = None if mu0 is None else np.ascontiguousarray(mu0, dtype=np.float64)
        check(self._lib.vampomi_pcg(self.ctx, _dp(v), None if m0 is None else _dp(m0), tau, gam2,
                                    1 if onsager else 0, max_iter, tol, _dp(mu), C.byref(it), MEM_HOST))
        return mu[: self.M], it.value

    def test_metrics(self, est: np.ndarray):
        """--run-mode test row (src/main_meth.cpp:165-199) for one estimate slice
        (x1_hat / sqrt(N)) on this (test) data set: (R2 test, squared z correlation)."""
        est = np.ascontiguousarray(est, dtype=np.float64)
        if est.shape != (self.M,):
            raise ValueError("estimate slice must have M entries")
        r2, c2 = C.c_double(), C.c_double()
        check(self._lib.vampomi_test_metrics(self.ctx, _dp(est), C.byref(r2), C.byref(c2), MEM_HOST))
        return r2.value, c2.value

    test_metrics.__test__ = False

    def assoc_loo(self, est: np.ndarray, mem_device: bool = False):
        """--pval-method loo (src/main_meth.cpp:245-264, src/data.cpp:385-417).
        est: this shard's estimate-file slice (x1_hat / sqrt(N)).  COLLECTIVE.
        Returns (pvals (M), stats (M, 5): sumx sumsqx sumxy sumy sumsqy)."""
        est = np.ascontiguousarray(est, dtype=np.float64)
        if est.shape != (self.M,):
            raise ValueError("estimate slice must have M entries")
        pv = np.zeros(max(self.M, 1))
        st = np.zeros((max(self.M, 1), 5))
        check(self._lib.vampomi_assoc_loo(self.ctx, _dp(est), _dp(pv), _dp(st), MEM_HOST))
        return pv[: self.M], st[: self.M]

    def assoc_se(self, r1: np.ndarray, gam1: float) -> np.ndarray:
        """--pval-method se (src/main_meth.cpp:218-242)."""
        r1 = np.ascontiguousarray(r1, dtype=np.float64)
        pv = np.zeros(max(self.M, 1))
        check(self._lib.vampomi_assoc_se(self.ctx, _dp(r1), gam1, _dp(pv), MEM_HOST))
        return pv[: self.M]

    def update_prior(self, r1: np.ndarray, gam1: float, probs, vars_scaled, EM_max_iter: int = 1,
                     EM_err_thr: float = 1e-2, learn_vars: int = 1, merge_vars_thr: float = 0.5):
        """vamp::updatePrior (src/vamp.cpp:531-643); vars multiplied by N. Returns (probs, vars)."""
        r1 = np.ascontiguousarray(r1, dtype=np.float64)
        L = C.c_int(len(probs))
        pr = np.zeros(MAX_L)
        va_ = np.zeros(MAX_L)
        pr[: L.value] = probs
        va_[: L.value] = vars_scaled
        check(self._lib.vampomi_update_prior(self.ctx, _dp(r1), gam1, C.byref(L), _dp(pr), _dp(va_), EM_max_iter,
                                             EM_err_thr, learn_vars, merge_vars_thr, MEM_HOST))
        return pr[: L.value].copy(), va_[: L.value].copy()

    def denoise_bin(self, p1: np.ndarray, tau1: float):
        """g1_bin_class / g1d_bin_class over the phenotype (src/vamp_probit.cpp:469-488): (z1, sum of g1d)."""
        p1 = np.ascontiguousarray(p1, dtype=np.float64)
        z = np.zeros(self.N)
        sd = C.c_double()
        check(self._lib.vampomi_denoise_bin(self.ctx, _dp(p1), tau1, _dp(z), C.byref(sd), MEM_HOST))
        return z, sd.value

    def denoise(self, r1: np.ndarray, gam1: float, probs: Sequence[float], vars_scaled: Sequence[float]):
        """(g1(r1), g1d(r1), sum of g1d over ranks); vars already multiplied by N."""
        r1 = np.ascontiguousarray(r1, dtype=np.float64)
        L = len(probs)
        pr = np.ascontiguousarray(probs, dtype=np.float64)
        va = np.ascontiguousarray(vars_scaled, dtype=np.float64)
        x1 = np.zeros(max(self.M, 1))
        x1d = np.zeros(max(self.M, 1))
        s = C.c_double()
        check(self._lib.vampomi_denoise(self.ctx, _dp(r1), gam1, _dp(pr), _dp(va), L, _dp(x1), _dp(x1d),
                                        C.byref(s), MEM_HOST))
        return x1[: self.M], x1d[: self.M], s.value

    # -- measurement --
    def kernel_name(self, which: int, K: int, mode: int = 0) -> str:
        """rocprofv3 name of the kernel this context launches for pass ``which``
        (0 A.x, 1 A^T.u, 2 association test, 3 one-pass CG operator under the
        context's plan)
        with K right-hand sides, under its current variant settings."""
        buf = C.create_string_buffer(256)
        check(self._lib.vampomi_dev_kernel_name(self.ctx, which, K, mode, buf, 256))
        return buf.value.decode()

    def op_apply(self, ar, p, diag: float, tau: float, gam2: float, z=None, qo=None, beta=None):
        """Development hook: one application of the one-pass CG operator on K <= 2
        systems (vampomi_dev_op_apply): returns (d, A d, <d, p>) for
        q = ar/diag [+ beta*qo] and p [= z + beta*p]."""
        ar = np.ascontiguousarray(np.atleast_2d(ar), dtype=np.float64)
        p = np.ascontiguousarray(np.atleast_2d(p), dtype=np.float64)
        K = ar.shape[0]
        if ar.shape != (K, self.N) or p.shape != (K, self.M):
            raise ValueError("ar must be K x N and p K x M")
        fz = z is not None
        if fz:
            z = np.ascontiguousarray(np.atleast_2d(z), dtype=np.float64)
            qo = np.ascontiguousarray(np.atleast_2d(qo), dtype=np.float64)
            beta = np.ascontiguousarray(beta, dtype=np.float64)
        d = np.zeros((K, max(self.M, 1)))
        ad = np.zeros((K, self.N))
        dp = np.zeros(K)
        check(self._lib.vampomi_dev_op_apply(self.ctx, K, _dp(ar), _dp(qo) if fz else None, _dp(p),
                                             _dp(z) if fz else None, _dp(beta) if fz else None, diag, tau, gam2,
                                             _dp(d), _dp(ad), _dp(dp)))
        return d[:, : self.M], ad, dp

    def read_ceiling(self, reps: int = 9) -> dict:
        """The HBM read ceiling on this device for this shard (vampomi_dev_read_ceiling):
        a pure read stream of the resident matrix, the faster variant's median."""
        us, nb, var = C.c_double(), C.c_double(), C.c_int()
        check(self._lib.vampomi_dev_read_ceiling(self.ctx, int(reps), C.byref(us), C.byref(nb), C.byref(var)))
        return {"us_med": us.value, "bytes": nb.value, "GBs": nb.value / (us.value * 1e-6) / 1e9,
                "variant": ("lockstep 8-wave workgroups, one per CU", "1 MiB chunk per wave")[var.value]}

    def set_variant(self, which: int, variant: int):
        """Development hook: this context's kernel variant for pass ``which``."""
        check(self._lib.vampomi_dev_set_variant(self.ctx, which, variant))

    def all_ok(self, local_ok: bool) -> bool:
        """COLLECTIVE: True iff local_ok on every rank."""
        out = C.c_int()
        check(self._lib.vampomi_all_ok(self.ctx, 1 if local_ok else 0, C.byref(out)))
        return bool(out.value)

    def comm_abort(self):
        """Poison (loopback) / abort (RCCL) the job's communicator after a local failure."""
        check(self._lib.vampomi_comm_abort(self.ctx))

    def set_timing(self, on: bool = True, period: int = 1):
        """HIP-event timing of the A/A^T launches; period > 1 times one launch
        in `period` of each (kernel class, K) and counts it `period` times."""
        check(self._lib.vampomi_set_timing(self.ctx, (max(1, int(period)) if on else 0)))

    def stats(self) -> Stats:
        s = Stats()
        check(self._lib.vampomi_get_stats(self.ctx, C.byref(s)))
        return s

    def reset_stats(self):
        check(self._lib.vampomi_reset_stats(self.ctx))


@dataclass
class VampOptions:
    """Hyper-parameters of vamp::vamp (defaults: src/options.hpp:62-104)."""
    gam1: float = 1e-6
    h2: float = 0.5
    max_iter: int = 50
    CG_max_iter: int = 500
    CG_err_tol: float = 1e-5
    EM_max_iter: int = 1
    EM_err_thr: float = 1e-2
    rho: float = 0.5
    learn_vars: int = 1
    learn_prior_delay: int = 1
    stop_criteria_thr: float = 0.01
    merge_vars_thr: float = 0.5
    vars: Sequence[float] = (0, 1e-06, 6e-06, 3e-05, 2e-04, 1e-03, 6e-03, 3e-02, 2e-01, 1e+00)
    probs: Sequence[float] = (9.9e-01, 5e-03, 2.5e-03, 1.25e-03, 6.25e-04, 3.125e-04, 1.5625e-04, 7.8125e-05,
                              3.90625e-05, 3.90625e-05)
    seed: int = 0x5EED5EED
    out_dir: str = ""
    out_name: str = ""
    verbosity: int = 0
    batch_rhs: int = 4
    model: str = "linear"

    def to_struct(self) -> Params:
        p = Params()
        load().vampomi_params_default(C.byref(p))
        for k in ("gam1", "h2", "max_iter", "CG_max_iter", "CG_err_tol", "EM_max_iter", "EM_err_thr", "rho",
                  "learn_vars", "learn_prior_delay", "stop_criteria_thr", "merge_vars_thr", "seed", "verbosity",
                  "batch_rhs"):
            setattr(p, k, getattr(self, k))
        if len(self.vars) != len(self.probs) or not 1 <= len(self.vars) <= MAX_L:
            raise ValueError("vars and probs must have the same length (1..64)")
        p.L = len(self.vars)
        for j, (v, q) in enumerate(zip(self.vars, self.probs)):
            p.vars[j] = v
            p.probs[j] = q
        self._keep = [self.out_dir.encode(), self.out_name.encode(), self.model.encode()]
        p.out_dir, p.out_name, p.model = self._keep
        return p


class Vamp:
    """The reference's ``class vamp``: ``Vamp(data, opts).infere(...)``."""

    def __init__(self, data: Data, opts: Optional[VampOptions] = None, true_signal: Optional[np.ndarray] = None,
                 x1hat_init: Optional[np.ndarray] = None):
        self.data = data
        self.opts = opts or VampOptions()
        self.true_signal = None if true_signal is None else np.ascontiguousarray(true_signal, dtype=np.float64)
        self.x1hat_init = None if x1hat_init is None else np.ascontiguousarray(x1hat_init, dtype=np.float64)
        self._active = False

    def _prepare(self, keep_hist: bool):
        o, M = self.opts, self.data.M
        it = o.max_iter
        self.p = o.to_struct()
        if self.true_signal is not None:
            self.p.true_signal = self.true_signal.ctypes.data
        if self.x1hat_init is not None:
            self.p.x1hat_init = self.x1hat_init.ctypes.data
        self.cg = np.zeros(it, dtype=np.int32)
        self.ons = np.zeros(it, dtype=np.int32)
        self.Lh = np.zeros(it, dtype=np.int32)
        probit = o.model == "bin_class"
        self.params = np.zeros((it, 8 if probit else 5))
        self.metrics = np.zeros((it, 12 if probit else 6))
        self.prior = np.zeros((it, 1 + 2 * MAX_L)) if probit else None
        self.x1_final = np.zeros(max(M, 1))
        r = Result()
        ip = C.POINTER(C.c_int)
        r.cg_iters = self.cg.ctypes.data_as(ip)
        r.ons_iters = self.ons.ctypes.data_as(ip)
        r.L_hist = self.Lh.ctypes.data_as(ip)
        r.params = self.params.ctypes.data_as(C.POINTER(C.c_double))
        r.metrics = self.metrics.ctypes.data_as(C.POINTER(C.c_double))
        r.x1_final = self.x1_final.ctypes.data_as(C.POINTER(C.c_double))
        if self.prior is not None:
            r.prior_hist = self.prior.ctypes.data_as(C.POINTER(C.c_double))
        if keep_hist:
            self.x1_hist = np.zeros((it, max(M, 1)))
            self.r1_hist = np.zeros((it, max(M, 1)))
            r.x1_hist = self.x1_hist.ctypes.data_as(C.POINTER(C.c_double))
            r.r1_hist = self.r1_hist.ctypes.data_as(C.POINTER(C.c_double))
        self.r = r

    def infere(self, keep_hist: bool = False) -> np.ndarray:
        """Run vamp::infere to completion; returns what it returns (local slice):
        x1_hat / sqrt(N) for the linear model, x1_hat for bin_class."""
        self._prepare(keep_hist)
        check(load().vampomi_infere(self.data.ctx, C.byref(self.p), C.byref(self.r)))
        return self.x1_final[: self.data.M].copy()

    # step-wise API (one VAMP iteration per step)
    def begin(self, keep_hist: bool = False):
        self._prepare(keep_hist)
        check(load().vampomi_vamp_begin(self.data.ctx, C.byref(self.p), C.byref(self.r)))
        self._active = True

    def step(self) -> bool:
        s = C.c_int()
        check(load().vampomi_vamp_step(self.data.ctx, C.byref(s)))
        return bool(s.value)

    def step_phases(self):
        """The last step's (solves, whole step) seconds as the host sees them
        (vampomi_step_phases; the reference's "CG took" / "Total iteration time")."""
        a, b = C.c_double(), C.c_double()
        check(load().vampomi_step_phases(self.data.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def end(self) -> np.ndarray:
        check(load().vampomi_vamp_end(self.data.ctx))
        self._active = False
        return self.x1_final[: self.data.M].copy()

    @property
    def iterations_run(self) -> int:
        return self.r.iterations_run

    @property
    def a_passes(self):
        return self.r.a_passes_ref, self.r.a_passes_exec

    def summary(self) -> dict:
        n = self.r.iterations_run
        return {
            "iterations": n,
            "cg_iters": self.cg[:n].tolist(),
            "ons_iters": self.ons[:n].tolist(),
            "L": self.Lh[:n].tolist(),
            "params": self.params[:n].tolist(),
            "metrics": self.metrics[:n].tolist(),
            "a_passes_ref": self.r.a_passes_ref,
            "a_passes_exec": self.r.a_passes_exec,
            **({"prior": self.prior[:n].tolist()} if self.prior is not None else {}),
        }
