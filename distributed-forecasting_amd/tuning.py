"""Hyperparameter search as extra batch rows.

The reference's AutoML notebook searches Prophet's prior scales and
seasonality mode per series with ``ProphetHyperoptEstimator``
(notebooks/automl/22-09-26-06:54-Prophet-...py:109-123: search space
``changepoint_prior_scale`` ~ loguniform(-6.9, -0.69), ``seasonality_prior_scale``
and ``holidays_prior_scale`` ~ loguniform(-6.9, 2.3), ``seasonality_mode`` in
{additive, multiplicative}; metric ``smape``), one trial = one full Prophet fit
+ cross-validation on the CPU.  Here every (series, trial) pair is one row of
one batched launch: the rows of a trial share the series' grid and differ only
in their prior scales (``pf_problem.tau_series`` / ``sigmas_series``), so a
search of M trials over n series is M·n rows through the same K1 grid, K3 fit,
K4 forecast and K6 metrics kernels.  Seasonality mode is a kernel variant
(multiplicative / additive), so trials are grouped by mode, one engine each.

The sampler is the search space's own distributions drawn from a seeded numpy
``Generator`` (hyperopt's TPE adaptivity is not reproduced: with one batched
launch per fold, all trials of a round are evaluated at once).  The
``databricks.automl_runtime`` estimator is not in the reference tree, so its
fold layout is unpinned: folds follow UPSTREAM ``cross_validation``'s cutoffs
(``diagnostics.generate_cutoffs``) with the caller's horizon / period /
initial.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch

from . import batch as B
from . import diagnostics as D
from . import engine as E
from . import _lib as L

# notebooks/automl/22-09-26-06:54-Prophet-...py:112-117 (natural-log bounds)
SEARCH_SPACE = {
    "changepoint_prior_scale": (-6.9, -0.69),
    "seasonality_prior_scale": (-6.9, 2.3),
    "holidays_prior_scale": (-6.9, 2.3),
    "seasonality_mode": ("additive", "multiplicative"),
}
PRIOR_KEYS = ("changepoint_prior_scale", "seasonality_prior_scale", "holidays_prior_scale")


def sample_trials(n_trials: int, seed: int = 0, space: dict | None = None) -> list:
    """``n_trials`` points of the AutoML search space (loguniform prior
    scales, uniform choice of seasonality mode)."""
    space = SEARCH_SPACE if space is None else space
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_trials):
        tr = {}
        for k in PRIOR_KEYS:
            if k in space:
                lo, hi = space[k]
                tr[k] = float(np.exp(rng.uniform(lo, hi)))
        if "seasonality_mode" in space:
            modes = space["seasonality_mode"]
            tr["seasonality_mode"] = modes[int(rng.integers(len(modes)))]
        out.append(tr)
    return out


def expand_trials(n_series: int, trials: list, default_mode: str):
    """Row layout of a search: for each seasonality mode, the trial indices
    in that mode and the per-row (series, trial) index arrays, trial-major
    (row = j * n_series + s for the j-th trial of the group)."""
    groups = {}
    for j, tr in enumerate(trials):
        mode = tr.get("seasonality_mode", default_mode)
        if mode not in ("additive", "multiplicative"):
            raise ValueError(f"seasonality_mode {mode!r}")
        groups.setdefault(mode, []).append(j)
    layout = {}
    for mode, js in groups.items():
        tj = np.repeat(np.asarray(js, np.int64), n_series)
        si = np.tile(np.arange(n_series, dtype=np.int64), len(js))
        layout[mode] = (js, si, tj)
    return layout


def _row_priors(trials, tj, cfg):
    return {k: np.array([trials[j].get(k, getattr(cfg, k)) for j in tj], np.float64)
            for k in PRIOR_KEYS}


@dataclasses.dataclass
class SearchResult:
    trials: list
    metrics: np.ndarray        # [n_series, n_trials, len(L.CV_METRICS)]
    metric: str
    best_trial: np.ndarray     # [n_series] trial index (lowest metric; NaN-safe)
    best_params: list          # [n_series] dict

    def best_fit(self, engine_or_device, fit_ds, Y, series_ids=None) -> dict:
        """Refit every series on its full history with its best trial (one
        launch per seasonality mode).  Returns {mode: (series indices,
        FittedBatch)}."""
        dev = engine_or_device.device if isinstance(engine_or_device, E.Engine) \
            else int(engine_or_device)
        base = engine_or_device.config if isinstance(engine_or_device, E.Engine) \
            else E.ProphetConfig.reference()
        Yt = Y if isinstance(Y, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(Y, np.float64))
        out = {}
        modes = np.array([p.get("seasonality_mode", base.seasonality_mode)
                          for p in self.best_params])
        for mode in np.unique(modes):
            idx = np.flatnonzero(modes == mode)
            eng = E.Engine(dev, dataclasses.replace(base, seasonality_mode=str(mode)))
            pri = {k: np.array([self.best_params[i].get(k, getattr(base, k)) for i in idx])
                   for k in PRIOR_KEYS}
            sid = None if series_ids is None else np.asarray(series_ids)[idx]
            rows = torch.from_numpy(idx).to(Yt.device)
            fb = B.FittedBatch.fit_dense(eng, fit_ds, Yt[rows], series_ids=sid, priors=pri)
            out[str(mode)] = (idx, fb)
        return out


def hyperparameter_search(device: int, fit_ds, Y, trials: list, *, metric: str = "smape",
                          base_config: E.ProphetConfig | None = None,
                          horizon_days: float = 90, period_days: float = 360,
                          initial_days: float = 730, seed: int = 0) -> SearchResult:
    """Evaluate every trial on every row of ``Y`` ([n, T] on the shared date
    grid ``fit_ds``) by cross-validation, all (series, trial) pairs of one
    seasonality mode batched into the same launches.  Returns the metric
    table and each series' best trial (lowest ``metric``)."""
    if metric not in L.CV_METRICS:
        raise ValueError(f"metric must be one of {L.CV_METRICS}")
    base = base_config or E.ProphetConfig.reference()
    fit_ds = np.asarray(fit_ds, np.int64)
    Yt = Y if isinstance(Y, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(Y, np.float64))
    Yt = Yt.to(torch.device("cuda", device), torch.float64)
    n = Yt.shape[0]
    M = len(trials)
    if M == 0:
        raise ValueError("no trials")
    met = np.full((n, M, len(L.CV_METRICS)), np.nan)
    seasons = base.seasons(int(fit_ds[0]), int(fit_ds[-1]), B.min_positive_diff(fit_ds))
    for mode, (js, si, tj) in expand_trials(n, trials, base.seasonality_mode).items():
        eng = E.Engine(device, dataclasses.replace(base, seasonality_mode=mode))
        rows = Yt[torch.from_numpy(si).to(Yt.device)]
        m = D.cv_metrics_device(eng, fit_ds, rows, horizon_days=horizon_days,
                                period_days=period_days, initial_days=initial_days,
                                seasons=seasons, coverage=(metric == "coverage"), seed=seed,
                                priors=_row_priors(trials, tj, base)).cpu().numpy()
        met[si, tj] = m
    col = L.CV_METRICS.index(metric)
    score = met[:, :, col]
    if metric == "coverage":      # closest to the nominal interval width
        score = np.abs(score - base.interval_width)
    score = np.where(np.isnan(score), np.inf, score)
    best = np.argmin(score, axis=1)
    params = [dict(trials[j]) for j in best]
    return SearchResult(list(trials), met, metric, best, params)
