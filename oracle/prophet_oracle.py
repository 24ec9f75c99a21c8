"""CPU oracle for the per-series Prophet fit + forecast hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker (or the timed CPU baseline) — never as the product path.  The product
path is the HIP engine in ``distributed-forecasting_amd/``; it fails loudly
when its shared library is missing.

What this restates
------------------
The reference (``/root/reference``) contains no arithmetic of its own for this
path: ``notebooks/prophet/02_training.py:162-205`` configures and calls
third-party Prophet (``fbprophet==0.7.1`` / ``prophet`` 1.0.x,
``requirements.txt:3-4``) whose MAP fit runs the Stan model ``prophet.stan``
through PyStan 2.19's L-BFGS.  None of that code is on disk here, so every
function below is a restatement of the PUBLISHED upstream algorithm
(Prophet 1.0 ``forecaster.py`` / ``diagnostics.py``, ``stan/unix/prophet.stan``,
Stan 2.19 ``optimization/bfgs*.hpp``), anchored on the reference's call sites.

Parity status
-------------------------------------
* PINNED by known-answer tests: the date grid
  (days since epoch, ``t``), changepoint placement (``linspace(...).round()``),
  CV cutoffs and percentile positions.
* PARITY UNPINNED for everything that needs Prophet/Stan to run (objective,
  L-BFGS trajectory, predict, uncertainty sampler): no Prophet, Stan or golden
  vectors exist in the reference or this container.  The objective is pinned
  against finite differences and the L-BFGS optimum against a scipy
  L-BFGS-B polish (certified optimum), as SURVEY.md §8c item 9 prescribes.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import pandas as pd

NS_PER_DAY = 86400 * 10**9
EPOCH_NS = 0  # 1970-01-01 in datetime64[ns]

# Prophet constructor arguments used by the reference
# (notebooks/prophet/02_training.py:162-169) + upstream defaults.
DEFAULT_CONFIG = dict(
    growth="linear",
    n_changepoints=25,
    changepoint_range=0.8,
    changepoint_prior_scale=0.05,
    seasonality_prior_scale=10.0,
    holidays_prior_scale=10.0,
    seasonality_mode="multiplicative",
    interval_width=0.95,
    uncertainty_samples=1000,
    yearly=(365.25, 10),
    weekly=(7.0, 3),
    daily=None,
)


# ----------------------------------------------------------------------------
# a1: setup_dataframe / initialize_scales (UPSTREAM forecaster.py)
# ----------------------------------------------------------------------------
@dataclass
class History:
    ds_ns: np.ndarray        # int64 ns of the non-NaN rows, sorted
    y: np.ndarray            # float64 raw y
    y_scaled: np.ndarray
    t: np.ndarray
    start_ns: int
    t_scale_ns: int
    y_scale: float
    history_dates_ns: np.ndarray   # sorted unique ds of ALL input rows
    cap_scaled: np.ndarray | None = None


def setup_history(ds_ns, y, cap=None) -> History:
    """``Prophet.fit`` → ``setup_dataframe(initialize_scales=True)``.

    Drop NaN y (``history = df[df['y'].notnull()]``), require >= 2 rows,
    sort by ds (stable, ``sort_values('ds')``), ``y_scale = max|y - 0|``
    (1 if 0), ``start = min ds``, ``t_scale = max ds - start``,
    ``t = (ds - start) / t_scale`` (numpy m8/m8 → double/double).
    Called from 02_training.py:172 (``model.fit(history_pd)``).
    """
    ds_ns = np.asarray(ds_ns, dtype=np.int64)
    y = np.asarray(y, dtype=np.float64)
    if np.isinf(y).any():
        raise ValueError("Found infinity in column y.")
    history_dates = np.unique(ds_ns)
    keep = ~np.isnan(y)
    ds_h, y_h = ds_ns[keep], y[keep]
    if ds_h.shape[0] < 2:
        raise ValueError("Dataframe has less than 2 non-NaN rows.")
    order = np.argsort(ds_h, kind="stable")
    ds_h, y_h = ds_h[order], y_h[order]
    y_scale = float(np.abs(y_h).max())
    if y_scale == 0:
        y_scale = 1.0
    start = int(ds_h[0])
    t_scale = int(ds_h[-1] - start)
    t = (ds_h - start).astype(np.float64) / np.float64(t_scale)
    cap_s = None
    if cap is not None:
        cap_h = np.asarray(cap, dtype=np.float64)[keep][order]
        cap_s = cap_h / y_scale
    return History(ds_h, y_h, y_h / y_scale, t, start, t_scale, y_scale,
                   history_dates, cap_s)


def t_of(ds_ns, start_ns, t_scale_ns):
    return (np.asarray(ds_ns, np.int64) - start_ns).astype(np.float64) / np.float64(t_scale_ns)


# ----------------------------------------------------------------------------
# a2: fourier_series / make_all_seasonality_features (UPSTREAM forecaster.py)
# ----------------------------------------------------------------------------
def days_since_epoch(ds_ns):
    """``(dates - datetime(1970,1,1)).dt.total_seconds().astype(float) / (3600*24.)``:
    pandas total_seconds = int64 ns / 1e9 (float64), then / 86400."""
    ns = np.asarray(ds_ns, dtype=np.int64) - EPOCH_NS
    return (ns / 1e9) / (3600 * 24.0)


def fourier_series(ds_ns, period, order):
    """Columns sin(2π(i+1)d/P), cos(2π(i+1)d/P) for i < order, interleaved
    (``for i in range(order) for fun in (sin, cos)``); argument evaluated
    left-to-right as ``2.0 * (i + 1) * np.pi * t / period``."""
    d = days_since_epoch(ds_ns)
    cols = []
    for i in range(order):
        arg = 2.0 * (i + 1) * np.pi * d / period
        cols.append(np.sin(arg))
        cols.append(np.cos(arg))
    return np.column_stack(cols)


def seasonality_blocks(cfg=None):
    """Ordered (name, period, order) list — Prophet adds yearly, weekly, daily
    in that order (``set_auto_seasonalities``)."""
    cfg = dict(DEFAULT_CONFIG if cfg is None else cfg)
    blocks = []
    for name in ("yearly", "weekly", "daily"):
        spec = cfg.get(name)
        if spec:
            blocks.append((name, float(spec[0]), int(spec[1])))
    return blocks


def make_features(ds_ns, cfg=None, holiday_cols=None):
    """X[T×F], prior scales, s_a, s_m (``make_all_seasonality_features`` +
    ``regressor_column_matrix``). Holiday indicator columns (config 5) are
    appended after the seasonalities with ``holidays_prior_scale``."""
    cfg = dict(DEFAULT_CONFIG if cfg is None else cfg)
    blocks = seasonality_blocks(cfg)
    feats, sig = [], []
    for _, period, order in blocks:
        feats.append(fourier_series(ds_ns, period, order))
        sig += [cfg["seasonality_prior_scale"]] * (2 * order)
    if holiday_cols is not None and holiday_cols.shape[1] > 0:
        feats.append(np.asarray(holiday_cols, np.float64))
        sig += [cfg["holidays_prior_scale"]] * holiday_cols.shape[1]
    if not feats:
        feats.append(np.zeros((len(ds_ns), 1)))
        sig.append(1.0)
    X = np.column_stack(feats)
    F = X.shape[1]
    mult = cfg["seasonality_mode"] == "multiplicative"
    s_m = np.full(F, 1.0 if mult else 0.0)
    s_a = np.full(F, 0.0 if mult else 1.0)
    return X, np.asarray(sig, np.float64), s_a, s_m


def holiday_features(ds_ns, holidays):
    """UPSTREAM make_holiday_features (Prophet 1.0 forecaster.py): for each
    holiday row and offset in [lower_window, upper_window], a column keyed
    '{holiday}_delim_{+|-}{|offset|}' set to 1 on the rows whose date
    (``dates.dt.date``) equals the holiday date + offset; columns sorted by key.
    Returns (X [T x n], keys)."""
    dates = pd.to_datetime(np.asarray(ds_ns, np.int64)).normalize()
    cols = {}
    for row in holidays.itertuples(index=False):
        dt = pd.Timestamp(row.ds).normalize()
        lw = int(getattr(row, "lower_window", 0))
        uw = int(getattr(row, "upper_window", 0))
        for offset in range(lw, uw + 1):
            occ = dt + pd.Timedelta(days=offset)
            key = "{}_delim_{}{}".format(row.holiday, "+" if offset >= 0 else "-", abs(offset))
            col = cols.setdefault(key, np.zeros(len(dates)))
            col[dates == occ] = 1.0
    keys = sorted(cols)
    X = np.column_stack([cols[k] for k in keys]) if keys else np.zeros((len(dates), 0))
    return X, keys


# ----------------------------------------------------------------------------
# a3: set_changepoints (UPSTREAM forecaster.py) + Stan get_changepoint_matrix
# ----------------------------------------------------------------------------
def changepoint_indices(T, n_changepoints=25, changepoint_range=0.8):
    """``hist_size = int(np.floor(T * changepoint_range))``; clamp n_cp to
    hist_size-1; ``np.linspace(0, hist_size-1, n_cp+1).round().astype(int)[1:]``.
    Returns the index array (possibly empty)."""
    hist_size = int(np.floor(T * changepoint_range))
    n_cp = n_changepoints
    if n_cp + 1 > hist_size:
        n_cp = hist_size - 1
    if n_cp > 0:
        idx = np.linspace(0, hist_size - 1, n_cp + 1).round().astype(int)
        return idx[1:]
    return np.zeros(0, dtype=int)


def changepoints_t(hist: History, n_changepoints=25, changepoint_range=0.8):
    idx = changepoint_indices(hist.t.shape[0], n_changepoints, changepoint_range)
    if idx.shape[0] == 0:
        return idx, np.array([0.0])  # dummy changepoint (S = 1)
    return idx, np.sort(hist.t[idx])


def changepoint_matrix(t, t_change):
    """Stan ``get_changepoint_matrix``: A[i,j] = 1{t_i >= t_change_j}."""
    return (np.asarray(t)[:, None] >= np.asarray(t_change)[None, :]).astype(np.float64)


# ----------------------------------------------------------------------------
# a4: growth inits (UPSTREAM forecaster.py)
# ----------------------------------------------------------------------------
def linear_growth_init(t, y_scaled):
    T = t[-1] - t[0]
    k = (y_scaled[-1] - y_scaled[0]) / T
    m = y_scaled[0] - k * t[0]
    return k, m


def logistic_growth_init(t, y_scaled, cap_scaled):
    i0, i1 = 0, len(t) - 1
    T = t[i1] - t[i0]
    C0, C1 = cap_scaled[i0], cap_scaled[i1]
    y0 = max(0.01 * C0, min(0.99 * C0, y_scaled[i0]))
    y1 = max(0.01 * C1, min(0.99 * C1, y_scaled[i1]))
    r0 = C0 / y0
    r1 = C1 / y1
    if abs(r0 - r1) <= 0.01:
        r0 = 1.05 * r0
    L0 = np.log(r0 - 1)
    L1 = np.log(r1 - 1)
    m = L0 * T / (L0 - L1)
    k = (L0 - L1) / T
    return k, m


# ----------------------------------------------------------------------------
# a5: Stan model prophet.stan — log posterior (propto, no Jacobian) + gradient
# ----------------------------------------------------------------------------
GROWTH = {"linear": 0, "logistic": 1, "flat": 2}


@dataclass
class Problem:
    """The Stan data block (``dat`` in ``Prophet.fit``)."""
    t: np.ndarray
    y: np.ndarray            # y_scaled
    X: np.ndarray            # T × K
    t_change: np.ndarray     # S
    sigmas: np.ndarray
    s_a: np.ndarray
    s_m: np.ndarray
    tau: float
    growth: int = 0
    cap: np.ndarray | None = None
    A: np.ndarray = field(default=None, repr=False)

    def __post_init__(self):
        if self.A is None:
            self.A = changepoint_matrix(self.t, self.t_change)
        if self.cap is None:
            self.cap = np.zeros_like(self.t)

    @property
    def S(self):
        return len(self.t_change)

    @property
    def K(self):
        return self.X.shape[1]

    @property
    def P(self):
        return 3 + self.S + self.K


def unpack(theta, S):
    """Stan unconstrained parameter order: k, m, delta[S], log(sigma_obs), beta[K]."""
    k, m = theta[0], theta[1]
    delta = theta[2:2 + S]
    ls = theta[2 + S]
    beta = theta[3 + S:]
    return k, m, delta, ls, beta


def logistic_gamma(k, m, delta, t_change):
    S = len(t_change)
    k_s = np.concatenate(([k], k + np.cumsum(delta)))
    gamma = np.zeros(S)
    m_pr = m
    for i in range(S):
        gamma[i] = (t_change[i] - m_pr) * (1 - k_s[i] / k_s[i + 1])
        m_pr = m_pr + gamma[i]
    return gamma, k_s


def trend_scaled(pb: Problem, k, m, delta):
    if pb.growth == 0:
        return (k + pb.A @ delta) * pb.t + (m + pb.A @ (-pb.t_change * delta))
    if pb.growth == 1:
        gamma, _ = logistic_gamma(k, m, delta, pb.t_change)
        z = (k + pb.A @ delta) * (pb.t - (m + pb.A @ gamma))
        return pb.cap / (1.0 + np.exp(-z))
    return np.full_like(pb.t, m)


def log_posterior(pb: Problem, theta):
    """L(θ) with Stan ``propto`` dropping data-only constants:
    −k²/50 − m²/50 − Σ|δ|/τ − 2σ² − Σβ²/(2σ_f²) − T log σ − Σ r²/(2σ²)."""
    k, m, delta, ls, beta = unpack(np.asarray(theta, np.float64), pb.S)
    sigma = np.exp(ls)
    tr = trend_scaled(pb, k, m, delta)
    mu = tr * (1 + pb.X @ (beta * pb.s_m)) + pb.X @ (beta * pb.s_a)
    r = pb.y - mu
    T = len(pb.y)
    lp = -k * k / 50.0 - m * m / 50.0
    lp -= np.sum(np.abs(delta)) / pb.tau
    lp -= 2.0 * sigma * sigma
    lp -= np.sum(beta * beta / (2.0 * pb.sigmas * pb.sigmas))
    lp -= T * ls + np.sum(r * r) / (2.0 * sigma * sigma)
    return lp


def objective(pb: Problem, theta):
    """Minimisation objective used by Stan's optimizer: f = −L(θ), ∇f."""
    theta = np.asarray(theta, np.float64)
    k, m, delta, ls, beta = unpack(theta, pb.S)
    sigma = np.exp(ls)
    T = len(pb.y)
    xbm = pb.X @ (beta * pb.s_m)
    xba = pb.X @ (beta * pb.s_a)
    A = pb.A
    if pb.growth == 0:
        tr = (k + A @ delta) * pb.t + (m + A @ (-pb.t_change * delta))
    elif pb.growth == 1:
        gamma, k_s = logistic_gamma(k, m, delta, pb.t_change)
        Kt = k + A @ delta
        Mt = m + A @ gamma
        z = Kt * (pb.t - Mt)
        sg = 1.0 / (1.0 + np.exp(-z))
        tr = pb.cap * sg
    else:
        tr = np.full(T, m)
    mu = tr * (1 + xbm) + xba
    r = pb.y - mu
    rr = float(np.dot(r, r))
    inv_s2 = 1.0 / (sigma * sigma)
    L = (-k * k / 50.0 - m * m / 50.0 - np.sum(np.abs(delta)) / pb.tau
         - 2.0 * sigma * sigma - np.sum(beta * beta / (2.0 * pb.sigmas ** 2))
         - T * ls - rr * inv_s2 / 2.0)
    w = r * inv_s2                       # dL/dmu
    G = w * (1 + xbm)                    # dL/dtrend
    g = np.zeros_like(theta)
    S = pb.S
    if pb.growth == 0:
        g[0] = np.dot(G, pb.t) - k / 25.0
        g[1] = np.sum(G) - m / 25.0
        gd = A.T @ (G * pb.t) - pb.t_change * (A.T @ G)
    elif pb.growth == 1:
        a = G * pb.cap * sg * (1 - sg)
        dK = a * (pb.t - Mt)
        dM = -a * Kt
        # per-changepoint-segment sums; A is a step matrix → segment id
        seg = A.sum(axis=1).astype(int)
        PK = np.bincount(seg, weights=dK, minlength=S + 1)
        PM = np.bincount(seg, weights=dM, minlength=S + 1)
        bar_k = PK.copy()
        bar_m = PM.copy()
        for i in range(S - 1, -1, -1):
            bar_g = bar_m[i + 1]
            bar_m[i] += bar_m[i + 1]
            mpr = m + np.sum(gamma[:i])
            ki, ki1 = k_s[i], k_s[i + 1]
            bar_m[i] += bar_g * (-(1 - ki / ki1))
            bar_k[i] += bar_g * (-(pb.t_change[i] - mpr) / ki1)
            bar_k[i + 1] += bar_g * ((pb.t_change[i] - mpr) * ki / (ki1 * ki1))
        g[0] = np.sum(bar_k) - k / 25.0
        g[1] = bar_m[0] - m / 25.0
        gd = np.array([np.sum(bar_k[j + 1:]) for j in range(S)])
    else:
        g[0] = -k / 25.0
        g[1] = np.sum(G) - m / 25.0
        gd = np.zeros(S)
    g[2:2 + S] = gd - np.sign(delta) / pb.tau
    g[2 + S] = -T + rr * inv_s2 - 4.0 * sigma * sigma
    g[3 + S:] = pb.s_m * (pb.X.T @ (w * tr)) + pb.s_a * (pb.X.T @ w) - beta / pb.sigmas ** 2
    return -L, -g


# ----------------------------------------------------------------------------
# Full per-series problem construction (Prophet.fit minus the optimizer)
# ----------------------------------------------------------------------------
@dataclass
class FitSetup:
    hist: History
    problem: Problem
    cp_idx: np.ndarray
    theta0: np.ndarray
    constant: bool
    n_changepoints_requested: int


def build_problem(ds_ns, y, cfg=None, cap=None, holiday_cols_fn=None) -> FitSetup:
    cfg = dict(DEFAULT_CONFIG if cfg is None else cfg)
    hist = setup_history(ds_ns, y, cap=cap)
    hol = holiday_cols_fn(hist.ds_ns) if holiday_cols_fn else None
    X, sig, s_a, s_m = make_features(hist.ds_ns, cfg, hol)
    cp_idx, t_change = changepoints_t(hist, cfg["n_changepoints"], cfg["changepoint_range"])
    growth = GROWTH[cfg["growth"]]
    pb = Problem(hist.t, hist.y_scaled, X, t_change, sig, s_a, s_m,
                 float(cfg["changepoint_prior_scale"]), growth,
                 hist.cap_scaled)
    if growth == 0:
        k0, m0 = linear_growth_init(hist.t, hist.y_scaled)
    elif growth == 1:
        k0, m0 = logistic_growth_init(hist.t, hist.y_scaled, hist.cap_scaled)
    else:
        k0, m0 = 0.0, float(np.mean(hist.y_scaled))  # flat_growth_init
    theta0 = np.zeros(pb.P)
    theta0[0], theta0[1] = k0, m0
    theta0[2 + pb.S] = 0.0  # log(sigma_obs = 1)
    constant = bool(hist.y.min() == hist.y.max()) and growth in (0, 2)
    return FitSetup(hist, pb, cp_idx, theta0, constant, cfg["n_changepoints"])


# ----------------------------------------------------------------------------
# a7: predict (UPSTREAM forecaster.py: predict_trend, piecewise_linear,
#      predict_seasonal_components, yhat assembly)
# ----------------------------------------------------------------------------
def piecewise_linear(t, deltas, k, m, changepoint_ts):
    gammas = -changepoint_ts * deltas
    k_t = k * np.ones_like(t)
    m_t = m * np.ones_like(t)
    for s, t_s in enumerate(changepoint_ts):
        indx = t >= t_s
        k_t[indx] += deltas[s]
        m_t[indx] += gammas[s]
    return k_t * t + m_t


def piecewise_logistic(t, cap, deltas, k, m, changepoint_ts):
    k_cum = np.concatenate((np.atleast_1d(k), np.cumsum(deltas) + k))
    gammas = np.zeros(len(changepoint_ts))
    for i, t_s in enumerate(changepoint_ts):
        gammas[i] = ((t_s - m - np.sum(gammas)) * (1 - k_cum[i] / k_cum[i + 1]))
    k_t = k * np.ones_like(t)
    m_t = m * np.ones_like(t)
    for s, t_s in enumerate(changepoint_ts):
        indx = t >= t_s
        k_t[indx] += deltas[s]
        m_t[indx] += gammas[s]
    return cap / (1 + np.exp(-k_t * (t - m_t)))


@dataclass
class Params:
    k: float
    m: float
    delta: np.ndarray
    sigma_obs: float
    beta: np.ndarray


def params_from_theta(theta, S):
    k, m, delta, ls, beta = unpack(np.asarray(theta, np.float64), S)
    return Params(float(k), float(m), np.array(delta), float(np.exp(ls)), np.array(beta))


def make_future_dates(history_dates_ns, periods=90, freq_ns=NS_PER_DAY, include_history=True):
    """``make_future_dataframe(periods, freq='d', include_history=True)``:
    history_dates (all unique input ds) + ``periods`` dates after the last."""
    last = int(np.max(history_dates_ns))
    fut = last + freq_ns * np.arange(1, periods + 1, dtype=np.int64)
    if include_history:
        return np.concatenate((np.asarray(history_dates_ns, np.int64), fut))
    return fut


def predict_point(setup: FitSetup, params: Params, ds_ns, cfg=None, cap=None, holiday_cols_fn=None):
    """Point forecast columns: trend, multiplicative_terms, additive_terms,
    per-block components, yhat = trend·(1+mult) + add (all in y units)."""
    cfg = dict(DEFAULT_CONFIG if cfg is None else cfg)
    h = setup.hist
    t = t_of(ds_ns, h.start_ns, h.t_scale_ns)
    hol = holiday_cols_fn(ds_ns) if holiday_cols_fn else None
    X, _, s_a, s_m = make_features(ds_ns, cfg, hol)
    pb = setup.problem
    if pb.growth == 0:
        tr = piecewise_linear(t, params.delta, params.k, params.m, pb.t_change)
    elif pb.growth == 1:
        cap_s = np.asarray(cap, np.float64) / h.y_scale
        tr = piecewise_logistic(t, cap_s, params.delta, params.k, params.m, pb.t_change)
    else:
        tr = np.full_like(t, params.m)
    trend = tr * h.y_scale
    mult = X @ (params.beta * s_m)
    add = (X @ (params.beta * s_a)) * h.y_scale
    yhat = trend * (1 + mult) + add
    comps = {}
    col = 0
    for name, _, order in seasonality_blocks(cfg):
        w = np.zeros_like(params.beta)
        w[col:col + 2 * order] = 1.0
        c = X @ (params.beta * w)
        if cfg["seasonality_mode"] == "additive":
            c = c * h.y_scale
        comps[name] = c
        col += 2 * order
    return dict(t=t, trend=trend, multiplicative_terms=mult, additive_terms=add,
                yhat=yhat, X=X, **comps)


# ----------------------------------------------------------------------------
# a8: predict_uncertainty (UPSTREAM 0.7.1/1.0 sample_model /
#      sample_predictive_trend, Poisson-process trend changes) + nanpercentile
# ----------------------------------------------------------------------------
def sample_uncertainty(setup: FitSetup, params: Params, ds_ns, n_samples=1000,
                       interval_width=0.95, rng=None, cfg=None, cap=None,
                       return_samples=False):
    """Faithful per-sample loop: n ~ Poisson(S·(t_max−1)); new cp times
    1 + U·(t_max−1) sorted; λ = mean|δ| + 1e-8; δ_new ~ Laplace(0, λ);
    trend over concatenated changepoints; noise ~ N(0, σ_obs)·y_scale;
    yhat_s = trend_s·(1+Xb_m) + Xb_a + noise.  Percentiles with numpy
    'linear' interpolation at 100(1∓w)/2."""
    rng = np.random.default_rng() if rng is None else rng
    pt = predict_point(setup, params, ds_ns, cfg, cap)
    h, pb = setup.hist, setup.problem
    t = pt["t"]
    T_max = t.max()
    S_cp = len(pb.t_change)
    mult, add = pt["multiplicative_terms"], pt["additive_terms"]
    ys = np.empty((len(t), n_samples))
    trs = np.empty((len(t), n_samples))
    lam = np.mean(np.abs(params.delta)) + 1e-8
    for s in range(n_samples):
        n_changes = rng.poisson(S_cp * (T_max - 1)) if T_max > 1 else 0
        if n_changes > 0:
            cp_new = np.sort(1 + rng.random(n_changes) * (T_max - 1))
        else:
            cp_new = np.zeros(0)
        d_new = rng.laplace(0, lam, n_changes)
        cps = np.concatenate((pb.t_change, cp_new))
        ds_ = np.concatenate((params.delta, d_new))
        if pb.growth == 0:
            tr = piecewise_linear(t, ds_, params.k, params.m, cps)
        elif pb.growth == 1:
            tr = piecewise_logistic(t, np.asarray(cap) / h.y_scale, ds_, params.k, params.m, cps)
        else:
            tr = np.full_like(t, params.m)
        tr = tr * h.y_scale
        noise = rng.normal(0, params.sigma_obs, len(t)) * h.y_scale
        ys[:, s] = tr * (1 + mult) + add + noise
        trs[:, s] = tr
    lo_p = 100 * (1.0 - interval_width) / 2
    hi_p = 100 * (1.0 + interval_width) / 2
    out = dict(pt)
    out["yhat_lower"] = np.nanpercentile(ys, lo_p, axis=1)
    out["yhat_upper"] = np.nanpercentile(ys, hi_p, axis=1)
    out["trend_lower"] = np.nanpercentile(trs, lo_p, axis=1)
    out["trend_upper"] = np.nanpercentile(trs, hi_p, axis=1)
    if return_samples:
        out["yhat_samples"] = ys
        out["trend_samples"] = trs
    return out


def percentile_positions(n_samples=1000, interval_width=0.95):
    """numpy 'linear' method virtual index = q/100·(n−1)."""
    lo_p = 100 * (1.0 - interval_width) / 2
    hi_p = 100 * (1.0 + interval_width) / 2
    return lo_p / 100 * (n_samples - 1), hi_p / 100 * (n_samples - 1)


# ----------------------------------------------------------------------------
# a10: cross_validation cutoffs + performance_metrics (UPSTREAM diagnostics.py)
# ----------------------------------------------------------------------------
def generate_cutoffs(ds_ns, horizon_ns, initial_ns, period_ns):
    ds_ns = np.asarray(ds_ns, np.int64)
    dmin, dmax = int(ds_ns.min()), int(ds_ns.max())
    cutoff = dmax - horizon_ns
    if cutoff < dmin:
        raise ValueError("Less data than horizon.")
    result = [cutoff]
    while result[-1] >= dmin + initial_ns:
        cutoff -= period_ns
        if not np.any((ds_ns > cutoff) & (ds_ns <= cutoff + horizon_ns)):
            if cutoff > dmin:
                closest = int(ds_ns[ds_ns <= cutoff].max())
                cutoff = closest - horizon_ns
        result.append(cutoff)
    result = result[:-1]
    if len(result) == 0:
        raise ValueError("Less data than horizon after initial window.")
    return list(reversed(result))


def rolling_mean_by_h(x, h, w):
    hs, inv = np.unique(h, return_inverse=True)
    xs = np.bincount(inv, weights=x)
    ns = np.bincount(inv).astype(np.int64)
    trailing_i = len(hs) - 1
    x_sum, n_sum = 0.0, 0
    res_x = np.empty(len(hs))
    for i in range(len(hs) - 1, -1, -1):
        x_sum += xs[i]
        n_sum += ns[i]
        while n_sum >= w:
            excess_n = n_sum - w
            excess_x = excess_n * xs[i] / ns[i]
            res_x[trailing_i] = (x_sum - excess_x) / w
            x_sum -= xs[trailing_i]
            n_sum -= ns[trailing_i]
            trailing_i -= 1
    return hs[trailing_i + 1:], res_x[trailing_i + 1:]


def rolling_median_by_h(x, h, w):
    """UPSTREAM diagnostics.rolling_median_by_h (prophet 1.0): from the last
    horizon backwards, the median of the horizon's values extended with the
    preceding rows (sorted order) until w values; stop at the first horizon
    that cannot reach w."""
    hs = np.unique(h)
    res_h, res_x = [], []
    for i in range(len(hs) - 1, -1, -1):
        idx = np.flatnonzero(h == hs[i])
        xs = list(x[idx])
        nxt = idx[0] - 1
        while len(xs) < w and nxt >= 0:
            xs.append(x[nxt])
            nxt -= 1
        if len(xs) < w:
            break
        res_h.append(hs[i])
        res_x.append(np.median(xs))
    return np.array(res_h[::-1]), np.array(res_x[::-1])


def performance_metrics(y, yhat, horizon, rolling_window=0.1,
                        metrics=("mse", "rmse", "mae", "mape"), yhat_lower=None,
                        yhat_upper=None):
    """Rolling-by-horizon means as in UPSTREAM performance_metrics; MAPE is
    skipped when min|y| < 1e-8.  Returns dict metric -> per-horizon array."""
    y, yhat, horizon = map(np.asarray, (y, yhat, horizon))
    order = np.argsort(horizon, kind="stable")
    y, yhat, horizon = y[order], yhat[order], horizon[order]
    if yhat_lower is not None:
        yhat_lower = np.asarray(yhat_lower)[order]
        yhat_upper = np.asarray(yhat_upper)[order]
    n = len(y)
    w = int(rolling_window * n)
    w = max(w, 1)
    w = min(w, n)
    out = {}
    if "mse" in metrics or "rmse" in metrics:
        hs, v = rolling_mean_by_h((y - yhat) ** 2, horizon, w)
        out["horizon"] = hs
        if "mse" in metrics:
            out["mse"] = v
        if "rmse" in metrics:
            out["rmse"] = np.sqrt(v)
    if "mae" in metrics:
        hs, v = rolling_mean_by_h(np.abs(y - yhat), horizon, w)
        out["horizon"] = hs
        out["mae"] = v
    if "mape" in metrics and not (np.abs(y).min() < 1e-8):
        hs, v = rolling_mean_by_h(np.abs((y - yhat) / y), horizon, w)
        out["mape"] = v
    if "smape" in metrics:
        sape = 2 * np.abs(yhat - y) / (np.abs(y) + np.abs(yhat))
        hs, v = rolling_mean_by_h(sape, horizon, w)
        out["smape"] = v
    if "mdape" in metrics:
        hs, v = rolling_median_by_h(np.abs((y - yhat) / y), horizon, w)
        out["mdape"] = v
    if "coverage" in metrics and yhat_lower is not None:
        cov = ((y >= yhat_lower) & (y <= yhat_upper)).astype(np.float64)
        hs, v = rolling_mean_by_h(cov, horizon, w)
        out["coverage"] = v
    return out


def cv_metric_means(ds_ns, y, horizon_days=90, period_days=360, initial_days=730, cfg=None,
                    fit=None, metrics=("mse", "rmse", "mae", "mape", "smape")):
    """02_training.py:178-188 end to end on the CPU: cutoffs, one refit per
    fold (``fit(setup) -> theta``), point forecast of the fold's horizon,
    performance_metrics, mean over horizons.  Returns dict metric -> float
    (NaN where UPSTREAM skips the metric)."""
    ds_ns = np.asarray(ds_ns, np.int64)
    y = np.asarray(y, np.float64)
    H = int(horizon_days * NS_PER_DAY)
    cut = generate_cutoffs(ds_ns, H, int(initial_days * NS_PER_DAY), int(period_days * NS_PER_DAY))
    ys, fs, hs = [], [], []
    for c in cut:
        tr = ds_ns <= c
        te = (ds_ns > c) & (ds_ns <= c + H)
        st = build_problem(ds_ns[tr], y[tr], cfg)
        th = fit(st)
        pt = predict_point(st, params_from_theta(th, st.problem.S), ds_ns[te], cfg)
        ys.append(y[te]); fs.append(pt["yhat"]); hs.append(ds_ns[te] - c)
    pm = performance_metrics(np.concatenate(ys), np.concatenate(fs), np.concatenate(hs),
                             metrics=metrics)
    return {m: (float(np.mean(pm[m])) if m in pm else float("nan")) for m in metrics}
