"""ctypes binding of ``libprophet_hip.so`` (the C ABI in include/prophet_hip.h).

The library is built in-tree by ``build.py`` (hipcc --offload-arch=gfx950).
There is deliberately NO fallback: if the shared library is missing or cannot
be loaded, every engine entry point raises ``EngineUnavailable``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libprophet_hip.so")

PF_GROWTH = {"linear": 0, "logistic": 1, "flat": 2}
STATUS_NAMES = {0: "SUCCESS", 10: "ABSX", 20: "ABSF", 21: "RELF", 30: "ABSGRAD",
                31: "RELGRAD", 40: "MAXIT", -1: "LSFAIL", -2: "BADINIT", 50: "CONSTANT",
                60: "WARMUP", 70: "MAP"}
PF_ST_CONSTANT = 50

# Every symbol include/prophet_hip.h declares (checked by tests/test_host.py).
EXPORTED = ["pf_ctx_create", "pf_ctx_destroy", "pf_last_error", "pf_default_fit_opts",
            "pf_num_changepoints", "pf_build_grid", "pf_prepare", "pf_objective_grad",
            "pf_fit", "pf_predict", "pf_set_timing", "pf_read_timings", "pf_cv_metrics",
            "pf_hessian", "pf_prepare_ragged", "pf_build_grids", "pf_build_id", "pf_fit_forecast"]
PF_MAX_COMP = 32  # include/prophet_hip.h
PF_INTERVAL = {"exact": 0, "sample": 1}
PF_PREDICT_DET, PF_PREDICT_MC = 1, 2
PF_FF_ONLY_FUSED = 1
CV_METRICS = ["mse", "rmse", "mae", "mape", "smape", "coverage", "mdape"]


class EngineUnavailable(RuntimeError):
    pass


vp = ctypes.c_void_p
i32 = ctypes.c_int32


class PfSeason(ctypes.Structure):
    _fields_ = [("period", ctypes.c_double), ("order", i32), ("_pad", i32)]


class PfGrid(ctypes.Structure):
    _fields_ = [("T", i32), ("T_pad", i32), ("K", i32), ("S", i32),
                ("t", vp), ("XT", vp), ("t_change", vp), ("seg", vp), ("cp_first", vp)]


class PfProblem(ctypes.Structure):
    _fields_ = [("n_series", i32), ("growth", i32), ("tau", ctypes.c_double),
                ("grid", PfGrid),
                ("sigmas", vp), ("s_a", vp), ("s_m", vp), ("y_scaled", vp), ("cap_scaled", vp),
                ("fourier_orders", i32 * 3), ("season_mode", i32),
                ("tau_series", vp), ("sigmas_series", vp),
                ("n_grids", i32), ("grids", vp), ("grid_of", vp)]


class PfFitOpts(ctypes.Structure):
    _fields_ = [("init_alpha", ctypes.c_double), ("tol_obj", ctypes.c_double),
                ("tol_rel_obj", ctypes.c_double), ("tol_grad", ctypes.c_double),
                ("tol_rel_grad", ctypes.c_double), ("tol_param", ctypes.c_double),
                ("max_iter", i32), ("history", i32), ("polish", i32), ("polish_max_iter", i32),
                ("lbfgs_warmup", i32), ("lbfgs_warmup_evals", i32), ("tile_min_series", i32),
                ("polish_max_lag", i32), ("polish_lag_ratio", ctypes.c_double),
                ("polish_lam0", ctypes.c_double), ("lbfgs_warmup_ls_slack", i32)]


class PfPredictArgs(ctypes.Structure):
    _fields_ = [("n_series", i32), ("growth", i32), ("n_samples", i32), ("interval_method", i32),
                ("fg", PfGrid),
                ("s_a", vp), ("s_m", vp), ("theta", vp), ("y_scale", vp), ("cap_scaled", vp),
                ("interval_width", ctypes.c_double), ("seed", ctypes.c_uint64),
                ("yhat", vp), ("yhat_lower", vp), ("yhat_upper", vp),
                ("trend", vp), ("trend_lower", vp), ("trend_upper", vp),
                ("mult_terms", vp), ("add_terms", vp),
                ("n_comp", i32), ("comp_col0", i32 * PF_MAX_COMP), ("comp_ncol", i32 * PF_MAX_COMP), ("comp", vp),
                ("series_id", vp),
                ("n_grids", i32), ("grids", vp), ("grid_of", vp), ("parts", i32)]


class PfCvArgs(ctypes.Structure):
    _fields_ = [("n_series", i32), ("n_rows", i32), ("n_groups", i32), ("window", i32),
                ("group_start", vp), ("y", vp), ("yhat", vp), ("yhat_lower", vp),
                ("yhat_upper", vp), ("metrics", vp), ("ld_y", i32), ("ld_f", i32),
                ("skip_mdape", i32)]


class PfKernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("ms", ctypes.c_float), ("grid", i32)]


_lib = None


def check_build_id(path: str = LIB_PATH, csrc: str | None = None, include: str | None = None) -> str:
    """Refuse a library that was not compiled from the sources next to it:
    its embedded PF_BUILD_ID must equal the hash of csrc/ + include/ (build.py).
    Returns the id.  Raises EngineUnavailable on a mismatch (a stale .so)."""
    from . import build as _build
    src = _build.source_hash(csrc or _build.CSRC, include or _build.INCLUDE)
    got = _build.embedded_id(path)
    if src is None:
        raise EngineUnavailable(f"engine sources not found next to {path}: cannot verify the build")
    if got != src:
        raise EngineUnavailable(
            f"{path} is stale: built from sources with id {got}, the sources on disk hash to "
            f"{src}; rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    return got


def load(path: str = LIB_PATH):
    """Load the HIP engine library (raises EngineUnavailable if absent, or if
    the in-tree library's build id does not match its sources)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise EngineUnavailable(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    if os.path.abspath(path) == LIB_PATH:
        check_build_id(path)
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime
        raise EngineUnavailable(f"cannot load {path}: {e}") from e
    lib.pf_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.pf_ctx_destroy.argtypes = [vp]
    lib.pf_last_error.argtypes = [vp]
    lib.pf_last_error.restype = ctypes.c_char_p
    lib.pf_build_id.argtypes = []
    lib.pf_build_id.restype = ctypes.c_char_p
    lib.pf_default_fit_opts.argtypes = [ctypes.POINTER(PfFitOpts)]
    lib.pf_default_fit_opts.restype = None
    lib.pf_num_changepoints.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
    lib.pf_build_grid.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.POINTER(PfSeason), ctypes.c_int,
                                  vp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                  vp, vp, vp, vp, vp, vp, ctypes.c_int, vp]
    lib.pf_prepare.argtypes = [vp, ctypes.c_int, ctypes.POINTER(PfGrid), ctypes.c_int,
                               vp, vp, vp, vp, vp, vp, vp, vp]
    lib.pf_build_grids.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(PfSeason), ctypes.c_int, ctypes.c_int,
                                   ctypes.c_double, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp, vp]
    lib.pf_prepare_ragged.argtypes = [vp, ctypes.c_int, ctypes.POINTER(PfGrid), ctypes.c_int,
                                      vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.pf_objective_grad.argtypes = [vp, ctypes.POINTER(PfProblem), vp, vp, vp, vp]
    lib.pf_hessian.argtypes = [vp, ctypes.POINTER(PfProblem), vp, vp, vp]
    lib.pf_fit.argtypes = [vp, ctypes.POINTER(PfProblem), ctypes.POINTER(PfFitOpts),
                           vp, vp, vp, vp, vp, vp, vp]
    lib.pf_predict.argtypes = [vp, ctypes.POINTER(PfPredictArgs), vp]
    lib.pf_fit_forecast.argtypes = [vp, ctypes.POINTER(PfProblem), ctypes.POINTER(PfFitOpts),
                                    vp, vp, vp, vp, vp, vp, ctypes.POINTER(PfPredictArgs),
                                    ctypes.POINTER(PfCvArgs), ctypes.c_int, ctypes.POINTER(i32), vp]
    lib.pf_cv_metrics.argtypes = [vp, ctypes.POINTER(PfCvArgs), vp]
    lib.pf_set_timing.argtypes = [vp, ctypes.c_int]
    lib.pf_read_timings.argtypes = [vp, ctypes.POINTER(PfKernelTime), ctypes.c_int]
    for name in EXPORTED:
        if name not in ("pf_default_fit_opts", "pf_build_id"):
            getattr(lib, name).restype = getattr(lib, name).restype or ctypes.c_int
    _lib = lib
    return lib


def num_changepoints(T: int, n_changepoints: int = 25, changepoint_range: float = 0.8) -> int:
    """pf_num_changepoints (pure host arithmetic, no GPU)."""
    return int(load().pf_num_changepoints(int(T), int(n_changepoints), float(changepoint_range)))
