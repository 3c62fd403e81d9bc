"""ctypes binding of libdfm.so (the C ABI declared in include/dfm.h).

The library is built in-tree (``__graft_entry__.build()`` or ``make -C
dynamicfactormodels.jl_amd/csrc``).  There is no fallback: if the shared
object is missing or no GPU is visible, every entry point raises.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DFM_LIB_PATH: load another build of the same library (A/B timing of a
# variant built by the csrc Makefile's BUILD/LIB/EXTRA; tools/gpu_session.sh ab)
LIB_PATH = os.environ.get("DFM_LIB_PATH") or os.path.join(_HERE, "libdfm.so")

c_double_p = C.POINTER(C.c_double)
c_int32_p = C.POINTER(C.c_int32)
c_int64_p = C.POINTER(C.c_int64)
c_uint8_p = C.POINTER(C.c_uint8)


class dfm_stat(C.Structure):
    _fields_ = [("kind", C.c_int32), ("arg0", C.c_int32), ("arg1", C.c_int32), ("pad", C.c_int32)]


class dfm_window_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("length", C.c_int32), ("r", C.c_int32), ("crit", C.c_int32),
                ("kmax", C.c_int32), ("nbreaks", C.c_int32), ("breaks", C.POINTER(C.c_int64))]


# (name, restype, argtypes) — one row per symbol of include/dfm.h
SIGNATURES = [
    ("dfm_ctx_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("dfm_ctx_destroy", C.c_int, [C.c_void_p]),
    ("dfm_last_error", C.c_char_p, [C.c_void_p]),
    ("dfm_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("dfm_ctx_synchronize", C.c_int, [C.c_void_p]),
    ("dfm_ctx_set_eig_params", C.c_int, [C.c_void_p, C.c_double, C.c_int, C.c_int]),
    ("dfm_ctx_enable_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("dfm_ctx_read_timing", C.c_int, [C.c_void_p, c_double_p, c_int64_p, C.c_int]),
    ("dfm_ctx_reset_timing", C.c_int, [C.c_void_p]),
    ("dfm_ctx_eig_stats", C.c_int, [C.c_void_p, c_int64_p, c_int64_p, c_int64_p]),
    ("dfm_ctx_rep_iters", C.c_int, [C.c_void_p, c_int64_p]),
    ("dfm_ctx_gemm_products", C.c_int, [C.c_void_p, c_int64_p]),
    ("dfm_ctx_set_value_tol", C.c_int, [C.c_void_p, C.c_double]),
    ("dfm_kernel_class_name", C.c_char_p, [C.c_int]),
    ("dfm_pca", C.c_int, [C.c_void_p, c_double_p, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                          c_double_p, c_double_p, c_double_p, c_double_p]),
    ("dfm_full_spectrum_max", C.c_int, []),
    ("dfm_gram_spectrum", C.c_int, [C.c_void_p, c_double_p, C.c_int64, C.c_int64, C.c_int64,
                                    c_double_p, c_double_p]),
    ("dfm_ic_sweep", C.c_int, [c_double_p, C.c_int, C.c_int, C.c_double, C.c_int64, C.c_int64,
                               C.c_double, c_double_p]),
    ("dfm_model_fit", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64,
                                c_double_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                C.c_int, C.POINTER(C.c_void_p)]),
    ("dfm_model_fit_breaks", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64,
                                       c_double_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                       C.c_int, c_int64_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("dfm_model_destroy", C.c_int, [C.c_void_p]),
    ("dfm_model_blocks", C.c_int, [C.c_void_p]),
    ("dfm_model_block", C.c_int, [C.c_void_p, C.c_int, c_int64_p, c_int64_p, c_double_p, c_double_p]),
    ("dfm_model_dims", C.c_int, [C.c_void_p, c_int64_p, c_int64_p, c_int64_p]),
    ("dfm_model_scalars", C.c_int, [C.c_void_p, c_int64_p, c_double_p, c_double_p, c_double_p]),
    ("dfm_model_read", C.c_int, [C.c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                 c_double_p, c_double_p, c_double_p, c_double_p, c_double_p]),
    ("dfm_bootstrap", C.c_int, [C.c_void_p, C.c_int, C.c_int64, c_int32_p, c_double_p,
                                C.POINTER(dfm_stat), C.c_int, c_double_p]),
    ("dfm_bootstrap_dev", C.c_int, [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.POINTER(dfm_stat), C.c_int, C.c_void_p]),
    ("dfm_bootstrap_multi", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int64, c_int32_p,
                                      c_double_p, C.POINTER(dfm_stat), C.c_int, c_double_p]),
    ("dfm_model_clone", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("dfm_normalize", C.c_int, [C.c_void_p, c_double_p, C.c_int64, C.c_int64, C.c_int64, c_double_p,
                                C.c_int64]),
    ("dfm_normalize_dev", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_int64]),
    ("dfm_stats_width", C.c_int64, [C.c_void_p, C.POINTER(dfm_stat), C.c_int]),
    ("dfm_model_set_batch", C.c_int, [C.c_void_p, C.c_int64]),
    ("dfm_model_set_mode", C.c_int, [C.c_void_p, C.c_int]),
    ("dfm_model_fact_block", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("dfm_chow_all", C.c_int, [C.c_void_p, C.c_int64, c_double_p, c_double_p, c_double_p]),
    ("dfm_chow", C.c_int, [C.c_void_p, C.c_int64, C.c_int64, c_double_p, c_double_p, c_double_p]),
    ("dfm_model_criterion", C.c_int, [C.c_void_p, C.c_int, c_double_p]),
    ("dfm_get_factors", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, c_double_p]),
    ("dfm_predict", C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, c_double_p]),
    ("dfm_windows", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64, c_double_p,
                              C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, c_int64_p,
                              c_double_p, c_double_p, c_double_p, c_double_p, c_double_p]),
    ("dfm_windows_dev", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                  C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, c_int64_p,
                                  c_double_p, c_double_p, c_double_p, c_double_p, c_double_p]),
    ("dfm_windows_forecast", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64, c_double_p,
                                       C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, c_int64_p,
                                       c_double_p, c_double_p]),
    ("dfm_windows_ex", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p,
                                 C.c_int64, C.c_int64, C.c_int64, C.c_int, C.POINTER(dfm_window_spec), C.c_int,
                                 c_int64_p, c_double_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                 c_double_p, c_double_p]),
    ("dfm_targeted_hard", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64,
                                    c_double_p, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                    C.c_double, c_double_p, c_uint8_p]),
    ("dfm_lasso_path", C.c_int, [C.c_void_p, c_double_p, c_double_p, c_uint8_p, C.c_int, c_double_p, C.c_int,
                                 C.c_int, C.c_double, c_double_p, c_double_p, C.POINTER(C.c_int)]),
    ("dfm_targeted_soft", C.c_int, [C.c_void_p, c_double_p, c_double_p, C.c_int, C.c_int64,
                                    c_double_p, C.c_int64, C.c_int64, C.c_int64, c_int32_p,
                                    C.c_int, C.c_double, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    c_double_p, c_double_p, c_double_p, c_double_p, c_uint8_p]),
    ("dfm_lasso_stats", C.c_int, [c_int64_p, C.c_int, C.c_int]),
]

# dfm_lasso_stats slots (include/dfm.h DFM_LASSO_STAT_*)
LASSO_STATS = ("launches", "relaunches", "timeouts", "task_timeouts", "done_timeouts", "pipe_timeouts",
               "budget_overruns", "recovered", "max_skew_us", "late_entries", "max_kernel_us",
               "max_host_us", "slow_launches", "wave_splits")

_lock = threading.Lock()
_lib = None
_shutdown = False


def _mark_shutdown():
    global _shutdown
    _shutdown = True


atexit.register(_mark_shutdown)


def shutting_down() -> bool:
    """True once the interpreter is exiting: handles are then left to the OS
    (the HIP runtime may already be tearing down)."""
    return _shutdown


class LibraryMissing(RuntimeError):
    pass


def load():
    """Load libdfm.so (once).  Raises LibraryMissing — never falls back."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc, gfx950). There is no CPU fallback.")
        # torch (device memory for the *_dev entry points, torch.distributed)
        # must bring up the HIP runtime before libdfm does: loaded the other
        # way round, torch's later device init reports no HIP GPUs
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
        return lib


def exported_symbols():
    return [s[0] for s in SIGNATURES]


def ptr(a):
    """double* of a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(c_double_p)
