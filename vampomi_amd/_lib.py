"""ctypes binding of libvampomi (include/vampomi.h).

The library is built in-tree (vampomi_amd/lib/libvampomi.so) by
``python -m vampomi_amd.build`` or ``__graft_entry__.build()``.  There is no
fallback: if the shared library is missing, importing the product path raises.

If PyTorch is importable it is imported first, so that the process has a
single HIP runtime (torch's libamdhip64.so.7 satisfies libvampomi's
dependency by SONAME; loading ours first would let torch load a second copy).
"""
from __future__ import annotations

import ctypes as C
import os

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the library itself
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# VAMPOMI_LIB: another in-tree build of the same library (timing experiments, tools/)
LIB_PATH = os.environ.get("VAMPOMI_LIB") or os.path.join(HERE, "lib", "libvampomi.so")
CLI_PATH = os.path.join(HERE, "bin", "main_meth.exe")

MAX_L = 64
UNIQUE_ID_BYTES = 128
MEM_HOST, MEM_DEVICE = 0, 1
GEN_GAUSS, GEN_METH = 0, 1

STATUS = {
    0: "OK", 1: "ERR_ARG", 2: "ERR_HIP", 3: "ERR_RCCL", 4: "ERR_IO",
    5: "ERR_NAN_PHEN", 6: "ERR_STATE", 7: "ERR_OOM", 8: "ERR_MODEL",
}


class VampomiError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


class ShardDesc(C.Structure):
    _fields_ = [("N", C.c_int64), ("Mt", C.c_int64), ("rank", C.c_int), ("nranks", C.c_int),
                ("device", C.c_int), ("comm_id", C.c_void_p), ("alpha_scale", C.c_double)]


class Params(C.Structure):
    _fields_ = [
        ("gam1", C.c_double), ("h2", C.c_double),
        ("max_iter", C.c_int), ("CG_max_iter", C.c_int),
        ("CG_err_tol", C.c_double),
        ("EM_max_iter", C.c_int),
        ("EM_err_thr", C.c_double), ("rho", C.c_double),
        ("learn_vars", C.c_int), ("learn_prior_delay", C.c_int),
        ("stop_criteria_thr", C.c_double), ("merge_vars_thr", C.c_double),
        ("L", C.c_int),
        ("vars", C.c_double * MAX_L), ("probs", C.c_double * MAX_L),
        ("seed", C.c_uint64),
        ("out_dir", C.c_char_p), ("out_name", C.c_char_p),
        ("verbosity", C.c_int),
        ("true_signal", C.c_void_p), ("x1hat_init", C.c_void_p),
        ("batch_rhs", C.c_int),
        ("model", C.c_char_p),
    ]


class Result(C.Structure):
    _fields_ = [
        ("iterations_run", C.c_int),
        ("cg_iters", C.POINTER(C.c_int)), ("ons_iters", C.POINTER(C.c_int)), ("L_hist", C.POINTER(C.c_int)),
        ("params", C.POINTER(C.c_double)), ("metrics", C.POINTER(C.c_double)),
        ("x1_hist", C.POINTER(C.c_double)), ("r1_hist", C.POINTER(C.c_double)),
        ("x1_final", C.POINTER(C.c_double)),
        ("probs_final", C.c_double * MAX_L), ("vars_final", C.c_double * MAX_L),
        ("L_final", C.c_int),
        ("a_passes_ref", C.c_int64), ("a_passes_exec", C.c_int64),
        ("prior_hist", C.POINTER(C.c_double)),
    ]


class KernelStat(C.Structure):
    _fields_ = [("launches", C.c_int64), ("ms_total", C.c_double), ("bytes_total", C.c_double),
                ("flops_total", C.c_double), ("timed", C.c_int64), ("ms_timed", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("ax", KernelStat), ("atx", KernelStat), ("ax_k", KernelStat * 4), ("atx_k", KernelStat * 4),
                ("a_passes_exec", C.c_int64), ("host_syncs", C.c_int64), ("loo", KernelStat),
                ("op", KernelStat), ("op_k", KernelStat * 4), ("coll", KernelStat)]


# exported symbol -> (restype, argtypes); also the list the ABI test checks
_D = C.POINTER(C.c_double)
_P = C.c_void_p
SIGNATURES = {
    "vampomi_abi_version": (C.c_int, []),
    "vampomi_last_error": (C.c_char_p, []),
    "vampomi_divide_work": (None, [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int64)]),
    "vampomi_comm_unique_id": (C.c_int, [_P]),
    "vampomi_open": (C.c_int, [C.POINTER(ShardDesc), C.POINTER(_P)]),
    "vampomi_close": (None, [_P]),
    "vampomi_shard_info": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "vampomi_sync": (C.c_int, [_P]),
    "vampomi_barrier": (C.c_int, [_P]),
    "vampomi_barrier_timeout": (C.c_int, [_P, C.c_double]),
    "vampomi_load_meth_file": (C.c_int, [_P, C.c_char_p]),
    "vampomi_load_meth_host": (C.c_int, [_P, _P, C.c_int64]),
    "vampomi_generate_meth": (C.c_int, [_P, C.c_uint64, C.c_int]),
    "vampomi_read_phen": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "vampomi_set_phen": (C.c_int, [_P, _P, C.c_int]),
    "vampomi_get_phen": (C.c_int, [_P, _P]),
    "vampomi_simulate_phen": (C.c_int, [_P, C.c_uint64, C.c_double, C.c_double, _P]),
    "vampomi_simulate_phen_binary": (C.c_int, [_P, C.c_uint64, C.c_double, C.c_double, _P]),
    "vampomi_get_marker_stats": (C.c_int, [_P, _P, _P]),
    "vampomi_read_markers": (C.c_int, [_P, C.c_int64, C.c_int64, _P]),
    "vampomi_ax": (C.c_int, [_P, _P, _P, C.c_int]),
    "vampomi_atx": (C.c_int, [_P, _P, _P, C.c_int]),
    "vampomi_lmmse_mult": (C.c_int, [_P, _P, C.c_double, C.c_double, _P, C.c_int]),
    "vampomi_pcg": (C.c_int, [_P, _P, _P, C.c_double, C.c_double, C.c_int, C.c_int, C.c_double, _P,
                              C.POINTER(C.c_int), C.c_int]),
    "vampomi_test_metrics": (C.c_int, [_P, _P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int]),
    "vampomi_assoc_loo": (C.c_int, [_P, _P, _P, _P, C.c_int]),
    "vampomi_assoc_se": (C.c_int, [_P, _P, C.c_double, _P, C.c_int]),
    "vampomi_update_prior": (C.c_int, [_P, _P, C.c_double, C.POINTER(C.c_int), _P, _P, C.c_int, C.c_double,
                                        C.c_int, C.c_double, C.c_int]),
    "vampomi_denoise_bin": (C.c_int, [_P, _P, C.c_double, _P, C.POINTER(C.c_double), C.c_int]),
    "vampomi_denoise": (C.c_int, [_P, _P, C.c_double, _P, _P, C.c_int, _P, _P, C.POINTER(C.c_double), C.c_int]),
    "vampomi_params_default": (None, [C.POINTER(Params)]),
    "vampomi_infere": (C.c_int, [_P, C.POINTER(Params), C.POINTER(Result)]),
    "vampomi_vamp_begin": (C.c_int, [_P, C.POINTER(Params), C.POINTER(Result)]),
    "vampomi_vamp_step": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "vampomi_step_phases": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "vampomi_vamp_end": (C.c_int, [_P]),
    "vampomi_set_timing": (C.c_int, [_P, C.c_int]),
    "vampomi_get_stats": (C.c_int, [_P, C.POINTER(Stats)]),
    "vampomi_reset_stats": (C.c_int, [_P]),
    "vampomi_dev_set_variant": (C.c_int, [_P, C.c_int, C.c_int]),
    "vampomi_dev_time_pass": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "vampomi_dev_read_ceiling": (C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                           C.POINTER(C.c_int)]),
    "vampomi_dev_kernel_name": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int]),
    "vampomi_dev_mem_plan": (C.c_int, [C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P]),
    "vampomi_dev_ax_plan": (C.c_int, [C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, C.c_char_p,
                                      C.c_int]),
    "vampomi_dev_op_plan": (C.c_int, [C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, C.c_char_p,
                                      C.c_int]),
    "vampomi_dev_op_lds": (C.c_int, [C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _P]),
    "vampomi_dev_op_apply": (C.c_int, [_P, C.c_int, _P, _P, _P, _P, _P, C.c_double, C.c_double, C.c_double, _P, _P,
                                       _P]),
    "vampomi_dev_op_timestamps": (C.c_int, [_P, _P, C.c_int, C.POINTER(C.c_int)]),
    "vampomi_all_ok": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int)]),
    "vampomi_comm_abort": (C.c_int, [_P]),
}

_lib = None


def load() -> C.CDLL:
    """Load libvampomi.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -m vampomi_amd.build`")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        # another build named by VAMPOMI_LIB (an earlier round's, for an A/B)
        # may lack entry points added since; the product library may not
        other = bool(os.environ.get("VAMPOMI_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if other and not hasattr(lib, name):
                continue
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(status: int) -> None:
    if status != 0:
        msg = load().vampomi_last_error()
        raise VampomiError(status, msg.decode() if msg else "")
