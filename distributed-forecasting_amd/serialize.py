"""Prophet-format JSON export/import of fits (optional part).

The reference logs each fitted model with ``mlflow.prophet.log_model``
(notebooks/prophet/02_training.py:193-196) and logs ``serialize.SIMPLE_ATTRIBUTES``
as run params (02_training.py:146-147, :175).  MLflow's prophet flavour stores
the model with UPSTREAM ``serialize.model_to_json``.  This module writes that
JSON layout from a fit made here, so real Prophet can load our fits wherever it
is installed.  ``json_to_record`` reads the same layout back into a
params-store record, so fits written by real Prophet can be served through
``ForecastStoreItemModel`` without refitting.

Layout followed: fbprophet 0.7.1 ``serialize.model_to_dict`` (the version
``requirements.txt:4`` pins).  Attribute groups: SIMPLE_ATTRIBUTES verbatim;
PD_SERIES (changepoints, history_dates, train_holiday_names) as
``to_json(orient='split', date_format='iso')``; PD_TIMESTAMP ``start`` as epoch
seconds; PD_TIMEDELTA ``t_scale`` as seconds; PD_DATAFRAME (holidays, history,
train_component_cols) as ``to_json(orient='table', index=False)``; NP_ARRAY
``changepoints_t`` as a list; ORDEREDDICT (seasonalities, extra_regressors) as
``[keys, dict]``; ``params`` as nested lists of shape (1, ...).  Prophet is not
installed in this image, so the layout is "parity unpinned": the tests check
our own round trip and the fields against the fit, not a load by real Prophet.
"""
from __future__ import annotations

import json
from io import StringIO

import numpy as np
import pandas as pd

from .forecaster import SIMPLE_ATTRIBUTES

PROPHET_VERSION = "0.7.1"
PD_SERIES = ["changepoints", "history_dates", "train_holiday_names"]
PD_DATAFRAME = ["holidays", "history", "train_component_cols"]


def _trend(params: dict, t: np.ndarray, t_change: np.ndarray, growth: str) -> np.ndarray | None:
    """UPSTREAM piecewise_linear / flat trend on the history grid (prophet.stan
    ``trend``, in y/y_scale units).  Logistic trend is omitted (returns None)."""
    k = float(params["k"][0][0])
    m = float(params["m"][0][0])
    if growth == "flat":
        return np.full(t.shape, m)
    if growth != "linear":
        return None
    delta = np.asarray(params["delta"][0], np.float64)
    A = (t[:, None] >= t_change[None, :]).astype(np.float64) if len(t_change) else np.zeros((len(t), 0))
    return (k + A @ delta) * t + (m + A @ (-t_change * delta))


def _component_cols(model) -> pd.DataFrame:
    """UPSTREAM regressor_column_matrix: one row per feature column (beta
    order: seasonal Fourier columns, then holiday columns), one 0/1 column per
    component."""
    comp_of = [name for name, props in model.seasonalities.items()
               for _ in range(2 * int(props["fourier_order"]))]
    spec = getattr(model._batch.fit.grid, "holidays", None) if model._batch is not None else None
    hol_cols = list(spec.names) if spec is not None else []
    cols = {name: [int(c == name) for c in comp_of] + [0] * len(hol_cols)
            for name in model.seasonalities}
    for h in (spec.holidays if spec is not None else ()):
        cols[h] = [0] * len(comp_of) + [int(c.split("_delim_")[0] == h) for c in hol_cols]
    if hol_cols:
        cols["holidays"] = [0] * len(comp_of) + [1] * len(hol_cols)
    row_comp = comp_of + ["holidays"] * len(hol_cols)
    for grp, mode in (("additive_terms", "additive"), ("multiplicative_terms", "multiplicative")):
        members = set(model.component_modes[mode])
        cols[grp] = [int(c in members) for c in row_comp]
    cols["extra_regressors_additive"] = [0] * (len(comp_of) + len(hol_cols))
    cols["extra_regressors_multiplicative"] = [0] * (len(comp_of) + len(hol_cols))
    return pd.DataFrame(cols)


def model_to_dict(model) -> dict:
    """UPSTREAM serialize.model_to_dict for a fitted ``forecaster.Prophet``."""
    if model.history is None or model._batch is None:
        raise ValueError("This can only be used to serialize models that have already been fit.")
    d = {a: getattr(model, a, None) for a in SIMPLE_ATTRIBUTES}
    for a in PD_SERIES:
        v = getattr(model, a, None)
        d[a] = None if v is None else pd.Series(v).to_json(orient="split", date_format="iso")
    d["start"] = model.start.timestamp()
    d["t_scale"] = model.t_scale.total_seconds()
    hist = model.history
    d["holidays"] = None if model.holidays is None else model.holidays.to_json(orient="table", index=False)
    d["history"] = hist.to_json(orient="table", index=False)
    d["train_component_cols"] = _component_cols(model).to_json(orient="table", index=False)
    d["changepoints_t"] = np.asarray(model.changepoints_t, np.float64).tolist()
    d["seasonalities"] = [list(model.seasonalities.keys()), model.seasonalities]
    d["extra_regressors"] = [[], {}]
    d["fit_kwargs"] = dict(model.fit_kwargs)
    params = {k: np.asarray(v, np.float64) for k, v in model.params.items()}
    if "t" in hist:
        tr = _trend(params, hist["t"].to_numpy(np.float64),
                    np.asarray(model.changepoints_t, np.float64), model.growth)
        if tr is not None:
            params["trend"] = tr[None, :]
    d["params"] = {k: v.tolist() for k, v in params.items()}
    d["__fbprophet_version"] = PROPHET_VERSION
    return d


def model_to_json(model) -> str:
    """UPSTREAM serialize.model_to_json."""
    return json.dumps(model_to_dict(model))


def json_to_record(text: str, keys=None) -> dict:
    """Prophet-format JSON -> params-store record of one series (the fields
    ``FittedBatch.to_record`` writes; theta = [k, m, delta, log sigma_obs, beta]).

    The record carries the model's growth, seasonality mode and interval
    width; ``ParamsStore.put_record`` refuses it when they differ from the
    store's configuration (an additive fit is never served as multiplicative).
    Only layouts the engine can serve are accepted: growth linear/flat/logistic
    (logistic: the serving input must carry ``cap``), one mode shared by every
    seasonality, seasonalities with their own Fourier columns (no conditions),
    holidays (columns rebuilt from the model's holidays frame), no extra
    regressors, MAP fits (``mcmc_samples == 0``)."""
    from .batch import holiday_record, series_id
    from .holidays import holiday_spec
    d = json.loads(text)
    if int(d.get("mcmc_samples") or 0) > 0:
        raise NotImplementedError("mcmc_samples > 0 fits cannot be served (MAP only)")
    growth = str(d.get("growth", "linear"))
    if growth not in ("linear", "flat", "logistic"):
        raise NotImplementedError(f"growth {growth!r} cannot be served")
    if d.get("logistic_floor"):
        raise NotImplementedError("logistic floor is not supported")
    names, seas = d["seasonalities"]
    if d.get("extra_regressors") and d["extra_regressors"][0]:
        raise NotImplementedError("extra regressors are not supported")
    for n in names:
        if seas[n].get("condition_name"):
            raise NotImplementedError("conditional seasonalities are not supported")
    mode = str(d.get("seasonality_mode", "additive"))
    modes = {str(seas[n].get("mode", mode)) for n in names}
    if len(modes) > 1 or (modes and modes.pop() != mode):
        raise NotImplementedError("seasonalities with their own mode (not seasonality_mode) "
                                  "cannot be served")
    p = d["params"]
    theta = np.concatenate([np.asarray(p["k"], np.float64).reshape(-1)[:1],
                            np.asarray(p["m"], np.float64).reshape(-1)[:1],
                            np.asarray(p["delta"], np.float64).reshape(-1),
                            np.log(np.asarray(p["sigma_obs"], np.float64).reshape(-1)[:1]),
                            np.asarray(p["beta"], np.float64).reshape(-1)])
    P_seas = sum(2 * int(seas[n]["fourier_order"]) for n in names)
    S = len(d["changepoints_t"])
    spec = None
    if d.get("holidays"):
        hdf = pd.read_json(StringIO(d["holidays"]), orient="table")
        cm = d.get("component_modes") or {}
        hmode = "multiplicative" if "holidays" in cm.get("multiplicative", []) else (
            "additive" if "holidays" in cm.get("additive", []) else mode)
        spec = holiday_spec(hdf, float(d.get("holidays_prior_scale", 10.0)), hmode)
    n_hol = spec.n if spec is not None else 0
    if theta.shape[0] - 3 - S != P_seas + n_hol:
        raise NotImplementedError("beta has columns beyond the seasonal Fourier features and "
                                  "holidays (extra regressors?): not importable")
    hd = pd.read_json(StringIO(d["history_dates"]), typ="series", orient="split")
    rec = {
        "growth": np.str_(growth),
        "seasonality_mode": np.str_(mode),
        "interval_width": np.float64(d.get("interval_width", 0.8)),
        "theta": theta[None, :],
        "y_scale": np.array([float(d["y_scale"])]),
        "f": np.array([np.nan]),
        "status": np.array([0], np.int32),
        "n_eval": np.array([0], np.int32),
        "t_change": np.asarray(d["changepoints_t"], np.float64),
        "start_ns": np.int64(round(float(d["start"]) * 1e9)),
        "t_scale_ns": np.int64(round(float(d["t_scale"]) * 1e9)),
        "history_dates": pd.to_datetime(hd).to_numpy("datetime64[ns]").astype(np.int64),
        "season_names": np.array(list(names)),
        "season_periods": np.array([float(seas[n]["period"]) for n in names]),
        "season_orders": np.array([int(seas[n]["fourier_order"]) for n in names], np.int64),
    }
    rec.update(holiday_record(spec))
    if keys is not None:
        rec["keys"] = np.asarray(keys, np.int64).reshape(1, -1)
        # same per-series Monte-Carlo stream as a fit made here (batch.series_id)
        rec["series_id"] = series_id(rec["keys"])
    return rec
