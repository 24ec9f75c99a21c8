"""ctypes binding for oracle/stan_lbfgs.c (Stan objective + L-BFGS restatement).

TEST INFRASTRUCTURE ONLY — see prophet_oracle.py header.  Builds
``oracle/_build/liborc_stan.so`` with gcc on first use if it is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import prophet_oracle as po

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liborc_stan.so")
_lib = None

# Stan termination codes (bfgs.hpp TERM_*) + engine extras
STATUS_NAMES = {0: "SUCCESS", 10: "ABSX", 20: "ABSF", 21: "RELF", 30: "ABSGRAD",
                31: "RELGRAD", 40: "MAXIT", -1: "LSFAIL", 50: "CONSTANT", -2: "BADINIT"}


class OrcProblem(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int), ("K", ctypes.c_int), ("S", ctypes.c_int),
                ("growth", ctypes.c_int),
                ("t", ctypes.c_void_p), ("y", ctypes.c_void_p), ("cap", ctypes.c_void_p),
                ("X", ctypes.c_void_p), ("t_change", ctypes.c_void_p),
                ("sigmas", ctypes.c_void_p), ("s_a", ctypes.c_void_p), ("s_m", ctypes.c_void_p),
                ("tau", ctypes.c_double)]


class OrcOpts(ctypes.Structure):
    _fields_ = [("init_alpha", ctypes.c_double), ("tol_obj", ctypes.c_double),
                ("tol_rel_obj", ctypes.c_double), ("tol_grad", ctypes.c_double),
                ("tol_rel_grad", ctypes.c_double), ("tol_param", ctypes.c_double),
                ("max_iter", ctypes.c_int), ("history", ctypes.c_int),
                ("c1", ctypes.c_double), ("c2", ctypes.c_double), ("min_alpha", ctypes.c_double),
                ("max_ls_its", ctypes.c_int), ("max_ls_restarts", ctypes.c_int)]


def build():
    os.makedirs(os.path.join(_HERE, "_build"), exist_ok=True)
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-std=c11", "-shared", "-o", _LIB_PATH,
                           os.path.join(_HERE, "stan_lbfgs.c"), "-lm"])


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "stan_lbfgs.c")
        if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_objective.restype = ctypes.c_int
        _lib.orc_lbfgs_fit.restype = ctypes.c_int
        _lib.orc_default_opts.restype = None
    return _lib


def default_opts(**over):
    o = OrcOpts()
    lib().orc_default_opts(ctypes.byref(o))
    for k, v in over.items():
        setattr(o, k, v)
    return o


class _Pinned:
    """Keeps numpy buffers alive for the duration of a C call."""

    def __init__(self, pb: po.Problem):
        self.arrs = dict(
            t=np.ascontiguousarray(pb.t, np.float64),
            y=np.ascontiguousarray(pb.y, np.float64),
            cap=np.ascontiguousarray(pb.cap, np.float64),
            X=np.ascontiguousarray(pb.X, np.float64),
            t_change=np.ascontiguousarray(pb.t_change, np.float64),
            sigmas=np.ascontiguousarray(pb.sigmas, np.float64),
            s_a=np.ascontiguousarray(pb.s_a, np.float64),
            s_m=np.ascontiguousarray(pb.s_m, np.float64),
        )
        a = self.arrs
        self.c = OrcProblem(len(pb.t), pb.X.shape[1], len(pb.t_change), int(pb.growth),
                            a["t"].ctypes.data, a["y"].ctypes.data, a["cap"].ctypes.data,
                            a["X"].ctypes.data, a["t_change"].ctypes.data,
                            a["sigmas"].ctypes.data, a["s_a"].ctypes.data, a["s_m"].ctypes.data,
                            float(pb.tau))

    def set_y(self, y):
        self.arrs["y"] = np.ascontiguousarray(y, np.float64)
        self.c.y = self.arrs["y"].ctypes.data


def objective(pb: po.Problem, theta):
    pin = _Pinned(pb)
    th = np.ascontiguousarray(theta, np.float64)
    g = np.zeros_like(th)
    f = ctypes.c_double()
    bad = lib().orc_objective(ctypes.byref(pin.c), th.ctypes.data_as(ctypes.c_void_p),
                              ctypes.byref(f), g.ctypes.data_as(ctypes.c_void_p))
    return f.value, g, bad


def lbfgs(pb: po.Problem, theta0, opts=None):
    """Stan-faithful L-BFGS from theta0. Returns (theta, f, status, n_iter, n_eval)."""
    pin = _Pinned(pb)
    opts = default_opts() if opts is None else opts
    th = np.array(theta0, dtype=np.float64, copy=True)
    f = ctypes.c_double()
    it, ne = ctypes.c_int(), ctypes.c_int()
    st = lib().orc_lbfgs_fit(ctypes.byref(pin.c), ctypes.byref(opts),
                             th.ctypes.data_as(ctypes.c_void_p), ctypes.byref(f),
                             ctypes.byref(it), ctypes.byref(ne))
    return th, f.value, st, it.value, ne.value


def fit_setup(setup: po.FitSetup, opts=None):
    """Prophet.fit's optimizer step for one series: constant series skip the
    optimizer (params = init, sigma_obs = 1e-9); otherwise Stan L-BFGS."""
    if setup.constant:
        th = setup.theta0.copy()
        th[2 + setup.problem.S] = np.log(1e-9)
        return th, float("nan"), 50, 0, 0
    return lbfgs(setup.problem, setup.theta0, opts)


def certify(pb: po.Problem, theta_start, ftol=1e-15, gtol=1e-10, maxiter=20000):
    """Certified optimum: scipy L-BFGS-B polish from a start point
    (SURVEY.md §8c item 9).  Returns (theta, f)."""
    from scipy.optimize import minimize

    def fg(x):
        f, g, _ = objective(pb, x)
        return f, g

    best_x = np.array(theta_start, np.float64)
    best_f = fg(best_x)[0]
    x = best_x.copy()
    for _ in range(3):
        r = minimize(fg, x, jac=True, method="L-BFGS-B",
                     options=dict(ftol=ftol, gtol=gtol, maxiter=maxiter, maxcor=20))
        if r.fun < best_f:
            best_x, best_f = r.x.copy(), float(r.fun)
        x = r.x
    return best_x, best_f


def hessian(pb: po.Problem, theta):
    """Exact Hessian of the smooth part of f (linear, flat, logistic growth) —
    orc_hessian (analytic, incl. the second derivatives through logistic_gamma)."""
    pin = _Pinned(pb)
    th = np.ascontiguousarray(theta, np.float64)
    P = th.shape[0]
    H = np.zeros((P, P))
    rc = lib().orc_hessian(ctypes.byref(pin.c), th.ctypes.data_as(ctypes.c_void_p),
                           H.ctypes.data_as(ctypes.c_void_p), None)
    if rc:
        raise ValueError(f"orc_hessian failed ({rc})")
    return H


def hessian_fd(pb: po.Problem, theta, h=1e-6):
    """Central differences of the smooth gradient (the check for ``hessian``)."""
    pin = _Pinned(pb)
    th = np.ascontiguousarray(theta, np.float64)
    P = th.shape[0]
    H = np.zeros((P, P))
    rc = lib().orc_hessian_fd(ctypes.byref(pin.c), th.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_double(h), H.ctypes.data_as(ctypes.c_void_p))
    if rc:
        raise ValueError(f"orc_hessian_fd failed ({rc})")
    return H


POLISH_LAM0 = 1e-2   # stan_lbfgs.c ORC_POLISH_LAM0 = pf_default_fit_opts().polish_lam0


def polish(pb: po.Problem, theta, max_it=20, damp=False, return_cert=False, lam0=None,
           lam_decay=0.1, alpha_first=1.0):
    """Exact-MAP proximal-Newton polish (engine extension; same algorithm as
    the HIP kernel).  ``damp``: Levenberg-Marquardt damping when the exact
    Hessian model is not positive definite, and (``lam0``, default
    POLISH_LAM0 with damping) a damped first step.  Returns (theta, f, n_newton,
    n_eval, n_solve[, certified])."""
    if lam0 is None:          # the engine's default: damped first step (with damping on)
        lam0 = POLISH_LAM0 if damp else 0.0
    pin = _Pinned(pb)
    th = np.array(theta, dtype=np.float64, copy=True)
    f = ctypes.c_double()
    nn, ne, ns, cert = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_polish_cfg2(ctypes.byref(pin.c), th.ctypes.data_as(ctypes.c_void_p), int(max_it),
                               int(bool(damp)), ctypes.c_double(lam0), ctypes.c_double(lam_decay),
                               ctypes.c_double(alpha_first), ctypes.byref(f), ctypes.byref(nn),
                               ctypes.byref(ne), ctypes.byref(ns), ctypes.byref(cert))
    if rc:
        raise ValueError(f"orc_polish failed ({rc})")
    out = (th, f.value, nn.value, ne.value, ns.value)
    return out + (bool(cert.value),) if return_cert else out


def fit_map(setup: po.FitSetup, opts=None, polish_it=100, damp=True):
    """Engine semantics on the CPU: Stan L-BFGS, then the exact-MAP polish
    (every growth mode; Levenberg-Marquardt damping where the Hessian model
    is not positive definite, as the kernel does)."""
    th, f, st, it, ne = fit_setup(setup, opts)
    if setup.constant:
        return th, f, st, it, ne, f
    th2, f2, nn, ne2, ns = polish(setup.problem, th, polish_it, damp=damp)
    return th2, f2, st, it, ne + ne2, f
