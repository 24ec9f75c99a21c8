"""Prophet-shaped model on the HIP engine (UPSTREAM ``prophet.Prophet``).

The reference constructs ``Prophet(interval_width=0.95, growth='linear',
daily_seasonality=False, weekly_seasonality=True, yearly_seasonality=True,
seasonality_mode='multiplicative')`` per group, then ``fit`` →
``make_future_dataframe(periods=90, freq='d', include_history=True)`` →
``predict`` (notebooks/prophet/02_training.py:162-172, 201-205; the PyFunc
calls ``predict`` on a loaded model, model_wrapper.py:58-61).  This class keeps
that surface; ``fit`` is a batch of one through the same kernels the batched
entry points use.

Supported: linear, flat and logistic growth (capacity column 'cap', floor 0),
holidays (frame with holiday / ds / lower_window / upper_window / prior_scale),
auto/True/False/int seasonalities
(yearly, weekly, daily), additive and multiplicative seasonality, MAP fit,
``uncertainty_samples`` up to 1024.  Not supported yet (raise
NotImplementedError): logistic floor, extra regressors, custom
seasonalities, user-specified changepoints, ``mcmc_samples > 0``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import batch as B
from . import engine as E
from . import holidays as H

# UPSTREAM serialize.SIMPLE_ATTRIBUTES (what 02_training.py:146-147 logs)
SIMPLE_ATTRIBUTES = [
    "growth", "n_changepoints", "specified_changepoints", "changepoint_range",
    "yearly_seasonality", "weekly_seasonality", "daily_seasonality", "seasonality_mode",
    "seasonality_prior_scale", "changepoint_prior_scale", "holidays_prior_scale",
    "mcmc_samples", "interval_width", "uncertainty_samples", "y_scale", "logistic_floor",
    "country_holidays", "component_modes",
]

_ENGINES: dict = {}


def default_device() -> int:
    if not torch.cuda.is_available():
        # No CPU path exists; make the failure explicit.
        raise RuntimeError("no GPU visible: the Prophet engine runs only on MI355X (HIP)")
    return torch.cuda.current_device()


def get_engine(config: E.ProphetConfig, device: int | None = None) -> E.Engine:
    dev = default_device() if device is None else int(device)
    key = (dev, tuple(sorted(config.__dict__.items(), key=lambda kv: kv[0])))
    eng = _ENGINES.get(key)
    if eng is None:
        eng = E.Engine(dev, config)
        _ENGINES[key] = eng
    return eng


class Prophet:
    """Drop-in for UPSTREAM ``prophet.Prophet`` (MAP path)."""

    def __init__(self, growth="linear", changepoints=None, n_changepoints=25,
                 changepoint_range=0.8, yearly_seasonality="auto", weekly_seasonality="auto",
                 daily_seasonality="auto", holidays=None, seasonality_mode="additive",
                 seasonality_prior_scale=10.0, holidays_prior_scale=10.0,
                 changepoint_prior_scale=0.05, mcmc_samples=0, interval_width=0.80,
                 uncertainty_samples=1000, stan_backend=None, *, device=None, seed=0,
                 fit_mode="map"):
        if growth not in ("linear", "flat", "logistic"):
            raise ValueError('Parameter "growth" should be "linear", "logistic" or "flat".')
        if changepoints is not None:
            raise NotImplementedError("user-specified changepoints are not supported yet")
        if holidays is not None:
            # UPSTREAM validate_inputs: checked now, columns built at fit
            H.holiday_spec(holidays, float(holidays_prior_scale))
        if mcmc_samples:
            raise NotImplementedError("mcmc_samples > 0 (full posterior) is not supported")
        if seasonality_mode not in ("additive", "multiplicative"):
            raise ValueError('seasonality_mode must be "additive" or "multiplicative"')
        self.growth = growth
        self.changepoints = None
        self.specified_changepoints = False
        self.n_changepoints = n_changepoints
        self.changepoint_range = changepoint_range
        self.yearly_seasonality = yearly_seasonality
        self.weekly_seasonality = weekly_seasonality
        self.daily_seasonality = daily_seasonality
        self.holidays = None if holidays is None else holidays.copy()
        self.train_holiday_names = None
        self.seasonality_mode = seasonality_mode
        self.seasonality_prior_scale = float(seasonality_prior_scale)
        self.holidays_prior_scale = float(holidays_prior_scale)
        self.changepoint_prior_scale = float(changepoint_prior_scale)
        self.mcmc_samples = 0
        self.interval_width = interval_width
        self.uncertainty_samples = uncertainty_samples
        self.logistic_floor = False
        self.country_holidays = None
        self.device = device
        self.seed = seed
        self.stan_backend = stan_backend
        if fit_mode not in E.FIT_MODES:
            raise ValueError(f"fit_mode must be one of {E.FIT_MODES}")
        # engine option (ProphetConfig.fit_mode): "map" (certified MAP),
        # "stan_map", or "stan" (stop where Stan's L-BFGS stops)
        self.fit_mode = fit_mode
        # set by fit
        self.history = None
        self.history_dates = None
        self.start = None
        self.t_scale = None
        self.y_scale = None
        self.changepoints_t = None
        self.seasonalities = {}
        self.component_modes = None
        self.params = {}
        self.fit_kwargs = {}
        self._batch = None

    # ------------------------------------------------------------- config
    def config(self) -> E.ProphetConfig:
        return E.ProphetConfig(
            growth=self.growth, n_changepoints=self.n_changepoints,
            changepoint_range=self.changepoint_range,
            yearly_seasonality=self.yearly_seasonality,
            weekly_seasonality=self.weekly_seasonality,
            daily_seasonality=self.daily_seasonality, seasonality_mode=self.seasonality_mode,
            seasonality_prior_scale=self.seasonality_prior_scale,
            holidays_prior_scale=self.holidays_prior_scale,
            changepoint_prior_scale=self.changepoint_prior_scale,
            interval_width=self.interval_width,
            uncertainty_samples=int(self.uncertainty_samples or 0), fit_mode=self.fit_mode)

    # ---------------------------------------------------------------- fit
    def fit(self, df: pd.DataFrame, **kwargs) -> "Prophet":
        """UPSTREAM Prophet.fit: MAP fit of one series (02_training.py:172)."""
        if self.history is not None:
            raise Exception("Prophet object can only be fit once. Instantiate a new object.")
        if "ds" not in df or "y" not in df:
            raise ValueError('Dataframe must have columns "ds" and "y" with the dates and values respectively.')
        history = df[df["y"].notnull()].copy()
        if history.shape[0] < 2:
            raise ValueError("Dataframe has less than 2 non-NaN rows.")
        all_ds = B.to_ns(df["ds"])
        self.history_dates = pd.Series(np.unique(all_ds).astype("datetime64[ns]"), name="ds")
        ds = B.to_ns(history["ds"])
        y = history["y"].to_numpy(np.float64)
        if not np.all(np.isfinite(y)):
            raise ValueError("Found infinity in column y.")
        order = np.argsort(ds, kind="stable")
        ds, y = ds[order], y[order]
        cap = None
        if self.growth == "logistic":
            # UPSTREAM setup_dataframe: capacities are required; floor is not
            # supported on this path (logistic_floor = False)
            if "cap" not in history:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            if "floor" in history:
                raise NotImplementedError("logistic floor is not supported on the GPU path")
            cap = history["cap"].to_numpy(np.float64)[order][None, :]
            if np.any(cap <= 0.0):
                raise ValueError("Cap must be greater than floor (which defaults to 0).")
        spec = None
        if self.holidays is not None and len(self.holidays):
            # Prophet 1.0: holiday columns follow seasonality_mode
            spec = H.holiday_spec(self.holidays, self.holidays_prior_scale, self.seasonality_mode)
            self.train_holiday_names = pd.Series(list(spec.holidays))
        eng = get_engine(self.config(), self.device)
        fb = B.FittedBatch.fit_dense(eng, ds, y[None, :], history_dates=all_ds,
                                     series_ids=np.array([0], np.int32), cap=cap, holidays=spec)
        self._attach(fb, history=history.iloc[order].reset_index(drop=True))
        self.fit_kwargs = dict(kwargs)
        return self

    def _attach(self, fb: B.FittedBatch, history=None):
        """Populate Prophet's public attributes from a fitted batch of one."""
        self._batch = fb
        g = fb.fit.grid
        self.start = pd.Timestamp(int(g.start_ns))
        self.t_scale = pd.Timedelta(int(g.t_scale_ns))
        self.y_scale = float(fb.fit.y_scale[0].item())
        th = fb.fit.theta[0].cpu().numpy()
        tc = g.t_change.cpu().numpy()
        S = int(tc.shape[0])
        K = th.shape[0] - 3 - S
        placed = getattr(g, "n_changepoints_placed", S)
        # UPSTREAM set_changepoints: with no changepoints placed the model
        # keeps the dummy changepoints_t = [0] (delta then has one column)
        self.changepoints_t = tc if placed > 0 else np.array([0.0])
        cp_idx = getattr(g, "cp_idx", None)
        if placed > 0 and cp_idx is not None and fb.fit_ds is not None:
            cp_ds = fb.fit_ds[cp_idx.cpu().numpy()[:placed]]
        else:
            cp_ds = np.array([], dtype=np.int64)
        self.changepoints = pd.Series(cp_ds.astype("datetime64[ns]"), name="ds")
        self.params = {"k": th[None, 0:1], "m": th[None, 1:2], "delta": th[None, 2:2 + S],
                       "sigma_obs": np.exp(th[None, 2 + S:3 + S]), "beta": th[None, 3 + S:3 + S + K]}
        mode = self.seasonality_mode
        self.seasonalities = {name: {"period": p, "fourier_order": o, "prior_scale":
                                     self.seasonality_prior_scale, "mode": mode,
                                     "condition_name": None} for name, p, o in g.seasons}
        names = [s[0] for s in g.seasons]
        hspec = getattr(g, "holidays", None)
        if hspec is not None:
            names += list(hspec.holidays)
            self.holidays_prior_scales = dict(zip(hspec.names, hspec.prior_scales))
        add = [] if mode == "multiplicative" else list(names)
        mul = list(names) if mode == "multiplicative" else []
        add += ["additive_terms", "extra_regressors_additive"]
        mul += ["multiplicative_terms", "extra_regressors_multiplicative"]
        (mul if mode == "multiplicative" else add).append("holidays")
        self.component_modes = {"additive": add, "multiplicative": mul}
        if history is not None:
            h = history.copy()
            h["floor"] = 0.0
            h["t"] = (B.to_ns(h["ds"]) - int(g.start_ns)) / float(int(g.t_scale_ns))
            h["y_scaled"] = h["y"] / self.y_scale
            if "cap" in h:
                h["cap_scaled"] = h["cap"] / self.y_scale
            self.history = h
        else:
            self.history = pd.DataFrame({"ds": self.history_dates})

    @property
    def fit_status(self) -> str:
        from ._lib import STATUS_NAMES
        return STATUS_NAMES.get(int(self._batch.fit.status[0].item()), "?")

    # ------------------------------------------------------------ predict
    def make_future_dataframe(self, periods, freq="D", include_history=True) -> pd.DataFrame:
        """UPSTREAM make_future_dataframe (02_training.py:202-204)."""
        if self.history_dates is None:
            raise Exception("Model has not been fit.")
        dates = B.future_dates(B.to_ns(self.history_dates), int(periods), freq, include_history)
        return pd.DataFrame({"ds": dates.astype("datetime64[ns]")})

    def predict(self, df: pd.DataFrame | None = None) -> pd.DataFrame:
        """UPSTREAM Prophet.predict: trend, components, MC intervals, yhat
        (columns and order as Prophet 1.0 with MAP; fp32 values)."""
        if self._batch is None:
            raise Exception("Model has not been fit.")
        if df is None:
            df = self.history
        if df.shape[0] == 0:
            raise ValueError("Dataframe has no rows.")
        if "ds" not in df:
            raise ValueError('Dataframe must have column "ds".')
        ds = B.to_ns(df["ds"])
        order = np.argsort(ds, kind="stable")
        ds = ds[order]
        cap = None
        if self.growth == "logistic":
            if "cap" not in df:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            cap = df["cap"].to_numpy(np.float64)[order]
        return predict_frame(self._batch, 0, ds, self.seasonality_mode, seed=self.seed,
                             n_samples=int(self.uncertainty_samples or 0), cap=cap)


def predict_frame(fb: B.FittedBatch, row: int, ds: np.ndarray, mode: str, seed: int = 0,
                  n_samples: int = 1000, out=None, Tf=None, cap=None) -> pd.DataFrame:
    """Prophet-1.0 column layout for series ``row`` of a fitted batch
    (logistic growth: ``cap`` on the sorted dates, echoed after 'trend')."""
    if out is None:
        Tf, out = fb.predict(ds, seed=seed, n_samples=n_samples, components=True,
                             cap=None if cap is None else np.asarray(cap)[None, :])
    host = {k: v[row, :Tf].cpu().numpy() for k, v in out.items()}
    names = [s[0] for s in fb.fit.grid.seasons]
    hspec = getattr(fb.fit.grid, "holidays", None)
    if hspec is not None and hspec.n:
        names += sorted(set(hspec.holidays)) + ["holidays"]
    cols = {"ds": ds.astype("datetime64[ns]"), "trend": host["trend"]}
    if cap is not None:
        cols["cap"] = np.asarray(cap, np.float64)
    cols["yhat_lower"] = host["yhat_lower"]
    cols["yhat_upper"] = host["yhat_upper"]
    cols["trend_lower"] = host["trend_lower"]
    cols["trend_upper"] = host["trend_upper"]
    # UPSTREAM regressor_column_matrix: crosstab columns sorted by name, then
    # the missing one of additive_terms / multiplicative_terms appended.
    comps = {"additive_terms": host["additive_terms"],
             "multiplicative_terms": host["multiplicative_terms"]}
    for nm in names:
        comps[nm] = host[nm]
    present = sorted(names + (["multiplicative_terms"] if mode == "multiplicative"
                              else ["additive_terms"]))
    missing = ["additive_terms"] if mode == "multiplicative" else ["multiplicative_terms"]
    for nm in present + missing:
        v = comps[nm]
        cols[nm] = v
        cols[nm + "_lower"] = v      # MAP: one parameter draw → lower == upper == mean
        cols[nm + "_upper"] = v
    cols["yhat"] = host["yhat"]
    return pd.DataFrame(cols)
