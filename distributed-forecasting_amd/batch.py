"""Batched fit / forecast of many series that share one date grid.

The reference fits one Prophet per (store, item) group inside a Spark
``applyInPandas`` call (notebooks/prophet/02_training.py:282-307).  Here the
groups are packed into *buckets* — series whose non-NaN history dates and
whose full date set (``history_dates``, NaN rows included) are identical —
and each bucket is one dense ``Y[n, T_pad]`` float64 tensor in HBM, fitted
and forecast by single kernel launches.

Series identity: ``series_id(keys)`` = low 32 bits of splitmix64 of the packed
(store, item) key.  It keys each series' Monte-Carlo RNG stream (so the
intervals of a series do not depend on which bucket or GPU it landed on) and
the GPU shard.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import engine as E

NS_PER_DAY = E.NS_PER_DAY


# ---------------------------------------------------------------------------
# keys
# ---------------------------------------------------------------------------
def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over uint64 (vectorised)."""
    z = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def pack_keys(keys: np.ndarray) -> np.ndarray:
    """[n, k] integer keys -> uint64 (store << 32 | item for k == 2)."""
    keys = np.asarray(keys)
    if keys.ndim == 1:
        keys = keys[:, None]
    out = np.zeros(keys.shape[0], dtype=np.uint64)
    for j in range(keys.shape[1]):
        col = keys[:, j].astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
        out = (out << np.uint64(32)) | col if j else col
    return out


def series_hash(keys: np.ndarray) -> np.ndarray:
    return splitmix64(pack_keys(keys))


def series_id(keys: np.ndarray) -> np.ndarray:
    """int32 RNG-stream key per series (bit pattern of the low 32 hash bits)."""
    return (series_hash(keys) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)


def shard_of(keys: np.ndarray, world_size: int) -> np.ndarray:
    """GPU shard of each series: splitmix64((store << 32) | item) mod G."""
    return (series_hash(keys) % np.uint64(max(1, world_size))).astype(np.int64)


# ---------------------------------------------------------------------------
# grid helpers (UPSTREAM setup_dataframe / make_future_dataframe)
# ---------------------------------------------------------------------------
def to_ns(ds) -> np.ndarray:
    """Any date-like column -> int64 nanoseconds since the epoch."""
    import pandas as pd
    arr = np.asarray(ds)
    if arr.dtype.kind == "M":
        return arr.astype("datetime64[ns]").astype(np.int64)
    return pd.to_datetime(pd.Series(ds)).values.astype("datetime64[ns]").astype(np.int64)


def future_dates(history_dates_ns: np.ndarray, periods: int, freq="D",
                 include_history: bool = True) -> np.ndarray:
    """UPSTREAM make_future_dataframe: ``periods`` dates after the last
    history date at ``freq`` (pandas offset alias), optionally prefixed by the
    history dates."""
    import pandas as pd
    h = np.unique(np.asarray(history_dates_ns, np.int64))
    last = pd.Timestamp(int(h[-1]))
    dates = pd.date_range(start=last, periods=periods + 1, freq=freq)
    dates = dates[dates > last][:periods]
    fut = dates.values.astype("datetime64[ns]").astype(np.int64)
    return np.concatenate((h, fut)) if include_history else fut


def min_positive_diff(ds_sorted: np.ndarray) -> int:
    d = np.diff(ds_sorted)
    d = d[d != 0]
    return int(d.min()) if d.size else 0


# ---------------------------------------------------------------------------
# buckets
# ---------------------------------------------------------------------------
@dataclass
class Bucket:
    fit_ds: np.ndarray          # sorted non-NaN dates [T] (duplicates kept)
    history_dates: np.ndarray   # sorted unique dates of all rows (NaN y included)
    Y: np.ndarray               # [n, T] float64, columns aligned with fit_ds
    members: np.ndarray         # positions in the caller's group list


def bucket_groups(ds_list, y_list) -> list:
    """Pack per-group (ds, y) arrays into buckets of identical grids.

    Per group (UPSTREAM setup_dataframe): rows with NaN y are dropped from
    the fit history but their dates stay in ``history_dates``; fewer than two
    non-NaN rows is Prophet's ValueError."""
    sig_to_bucket = {}
    parts = []
    last = None                 # (ds array, bucket) of the previous group: the common case
    for g, (ds, y) in enumerate(zip(ds_list, y_list)):
        ds = np.asarray(ds, dtype=np.int64)
        y = np.asarray(y, dtype=np.float64)
        ok = ~np.isnan(y)
        n_ok = int(ok.sum())
        if n_ok < 2:
            raise ValueError("Dataframe has less than 2 non-NaN rows.")
        strictly = ds.shape[0] < 2 or bool(np.all(ds[1:] > ds[:-1]))
        if strictly and n_ok == ds.shape[0]:
            # sorted, unique, no NaN: fit dates = history dates = ds
            if last is not None and last[0].shape == ds.shape and np.array_equal(last[0], ds):
                b = last[1]
                parts[b][2].append(y)
                parts[b][3].append(g)
                continue
            fds = hd = ds
            yv = y
        else:
            order = np.argsort(ds[ok], kind="stable")
            fds = ds[ok][order]
            hd = np.unique(ds)
            yv = y[ok][order]
        key = (fds.tobytes(), hd.tobytes())
        b = sig_to_bucket.get(key)
        if b is None:
            b = len(parts)
            sig_to_bucket[key] = b
            parts.append((fds, hd, [], []))
        parts[b][2].append(yv)
        parts[b][3].append(g)
        if fds is ds and hd is ds:
            last = (ds, b)
    return [Bucket(fds, hd, np.stack(ys), np.asarray(mem, dtype=np.int64))
            for fds, hd, ys, mem in parts]


def ragged_packs(buckets, config) -> list:
    """Group buckets (lists of bucket indices) whose grids can share one
    ragged launch: the same seasonalities under UPSTREAM's auto rules on each
    bucket's own history span and the same number of changepoints.  Staggered
    launch dates, gaps and different end dates then cost one launch per pack
    instead of one per distinct date set (02_training.py:277-307: every
    (store, item) group brings its own history)."""
    from . import _lib as L
    key_to_pack, packs = {}, []
    for b, bk in enumerate(buckets):
        fds = bk.fit_ds
        if fds.shape[0] < 2 or int(fds[-1] - fds[0]) <= 0:
            key = ("single", b)        # fit_dense raises Prophet's error for it
        else:
            seasons = config.seasons(int(fds[0]), int(fds[-1]), min_positive_diff(fds))
            S = max(1, L.num_changepoints(fds.shape[0], config.n_changepoints,
                                          config.changepoint_range))
            key = (tuple(seasons), S)
        p = key_to_pack.get(key)
        if p is None:
            key_to_pack[key] = p = len(packs)
            packs.append([])
        packs[p].append(b)
    return packs


# ---------------------------------------------------------------------------
# fitted batch
# ---------------------------------------------------------------------------
@dataclass
class GridSpec:
    """What a forecast needs from the fit grid (also what the params store
    persists): seasonality spec, time scaling and the changepoints."""
    seasons: list
    start_ns: int
    t_scale_ns: int
    t_change: torch.Tensor
    holidays: object = None     # HolidaySpec of the fit grid (None: no holiday columns)


def holiday_record(spec) -> dict:
    """HolidaySpec -> plain arrays for a params-store record (no pickles)."""
    if spec is None or spec.n == 0:
        return {}
    return {"hol_names": np.array(spec.names), "hol_prior_scales": np.array(spec.prior_scales, np.float64),
            "hol_holidays": np.array(spec.holidays),
            "hol_rows": np.array(spec.rows, np.int64).reshape(-1, 2),
            "hol_mode": np.str_(spec.mode)}


def holiday_from_record(rec: dict):
    """Inverse of ``holiday_record`` (None when the record has no holiday columns)."""
    from .holidays import HolidaySpec
    if "hol_names" not in rec:
        return None
    rows = tuple((int(j), int(d)) for j, d in np.asarray(rec["hol_rows"]).reshape(-1, 2))
    return HolidaySpec(tuple(str(s) for s in rec["hol_names"]),
                       tuple(float(v) for v in rec["hol_prior_scales"]),
                       tuple(str(s) for s in rec["hol_holidays"]), rows, str(rec["hol_mode"]))


def check_record_config(rec: dict, cfg) -> None:
    """A record is served only under the settings it was fitted with (the
    reference stores each run's full Prophet model: 02_training.py:193-196,
    loaded whole at model_wrapper.py:58).  Raises ValueError on a mismatch of
    growth, seasonality mode or interval width."""
    for field, want in (("growth", cfg.growth), ("seasonality_mode", cfg.seasonality_mode)):
        if field in rec and str(rec[field]) != str(want):
            raise ValueError(f"record was fitted with {field}={str(rec[field])!r}; the store/engine "
                             f"config has {field}={want!r}")
    if "interval_width" in rec and abs(float(rec["interval_width"]) - float(cfg.interval_width)) > 1e-12:
        raise ValueError(f"record interval_width={float(rec['interval_width'])} differs from the "
                         f"config's {cfg.interval_width}")


def _dense(A, n: int, T: int, T_pad: int, dev) -> torch.Tensor:
    """[n, T] numpy/tensor -> zero-padded [n, T_pad] float64 device tensor."""
    out = torch.zeros((n, T_pad), dtype=torch.float64, device=dev)
    if isinstance(A, torch.Tensor):
        out[:, :T] = A[:, :T].to(dev, torch.float64)
    else:
        out[:, :T] = E._to_device_async(np.broadcast_to(np.asarray(A, np.float64), (n, T)), dev)
    return out


class FittedBatch:
    """n series fitted on one shared grid (all tensors on one GPU)."""

    def __init__(self, engine: E.Engine, fit: E.FitResult, history_dates: np.ndarray,
                 fit_ds: np.ndarray | None = None, series_ids: np.ndarray | None = None):
        self.engine = engine
        self.fit = fit
        self.history_dates = np.asarray(history_dates, np.int64)
        self.fit_ds = fit_ds
        self.series_ids = None
        if series_ids is not None:
            self.series_ids = E._to_device_async(np.asarray(series_ids, dtype=np.int32),
                                                 fit.theta.device)

    @property
    def n(self) -> int:
        return int(self.fit.theta.shape[0])

    @classmethod
    def fit_dense(cls, engine: E.Engine, fit_ds: np.ndarray, Y, history_dates=None,
                  series_ids=None, polish: bool | None = None, seasons=None, cap=None,
                  holidays=None, priors=None) -> "FittedBatch":
        """Fit every row of Y ([n, T] numpy or device tensor, raw y) on the
        sorted date grid ``fit_ds`` (K1 grid + K2/K3 fit).  ``seasons``
        overrides the auto rules (CV folds reuse the parent's seasonalities,
        UPSTREAM diagnostics.prophet_copy); ``holidays`` (holidays.HolidaySpec)
        appends its indicator columns.  ``priors``: per-row prior scales,
        a dict of Engine.series_priors keyword arguments."""
        cfg = engine.config
        fit_ds = np.asarray(fit_ds, np.int64)
        T = fit_ds.shape[0]
        if T < 2:
            raise ValueError("Dataframe has less than 2 non-NaN rows.")
        start, t_scale = int(fit_ds[0]), int(fit_ds[-1] - fit_ds[0])
        if t_scale <= 0:
            raise ValueError("history must span more than one distinct date")
        if seasons is None:
            seasons = cfg.seasons(start, int(fit_ds[-1]), min_positive_diff(fit_ds))
        grid = E.build_grid(fit_ds, seasons, start_ns=start, t_scale_ns=t_scale,
                            n_changepoints=cfg.n_changepoints,
                            changepoint_range=cfg.changepoint_range, device=engine.device,
                            holidays=holidays)
        dev = torch.device("cuda", engine.device)
        n = int(Y.shape[0])
        Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device=dev)
        if isinstance(Y, torch.Tensor):
            Yd[:, :T] = Y[:, :T].to(dev, torch.float64)
        else:
            # pinned staging: the H2D runs asynchronously (no pageable stall)
            Yd[:, :T] = E._to_device_async(np.asarray(Y, dtype=np.float64), dev)
        capd = None
        if cfg.growth == "logistic":
            if cap is None:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            capd = _dense(cap, n, T, grid.T_pad, dev)
        pri = engine.series_priors(grid, n, **priors) if priors is not None else None
        fit = engine.fit(grid, Yd, polish=polish, cap=capd, priors=pri)
        hd = fit_ds if history_dates is None else history_dates
        return cls(engine, fit, np.unique(hd), fit_ds, series_ids)

    @classmethod
    def fit_forecast_dense(cls, engine: E.Engine, fit_ds: np.ndarray, Y, future_ds: np.ndarray, *,
                           history_dates=None, series_ids=None, seed: int = 0,
                           components: bool = False):
        """``fit_dense`` followed by ``predict(future_ds)`` through
        Engine.fit_forecast: one launch where the layout allows (each series'
        forecast rows run in its fit workgroup as soon as its fit ends), the
        same bits as the two calls.  Returns (batch, T, forecast dict)."""
        cfg = engine.config
        fit_ds = np.asarray(fit_ds, np.int64)
        T = fit_ds.shape[0]
        if T < 2:
            raise ValueError("Dataframe has less than 2 non-NaN rows.")
        start, t_scale = int(fit_ds[0]), int(fit_ds[-1] - fit_ds[0])
        if t_scale <= 0:
            raise ValueError("history must span more than one distinct date")
        seasons = cfg.seasons(start, int(fit_ds[-1]), min_positive_diff(fit_ds))
        grid = E.build_grid(fit_ds, seasons, start_ns=start, t_scale_ns=t_scale,
                            n_changepoints=cfg.n_changepoints,
                            changepoint_range=cfg.changepoint_range, device=engine.device)
        future_ds = np.asarray(future_ds, np.int64)
        fg = E.build_grid(future_ds, seasons, start_ns=start, t_scale_ns=t_scale,
                          changepoint_range=cfg.changepoint_range, t_change=grid.t_change,
                          device=engine.device)
        dev = torch.device("cuda", engine.device)
        n = int(Y.shape[0])
        Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device=dev)
        if isinstance(Y, torch.Tensor):
            Yd[:, :T] = Y[:, :T].to(dev, torch.float64)
        else:
            Yd[:, :T] = E._to_device_async(np.asarray(Y, dtype=np.float64), dev)
        sid = None if series_ids is None else \
            E._to_device_async(np.asarray(series_ids, dtype=np.int32), dev)
        fit, out, _, _ = engine.fit_forecast(grid, Yd, fg, seed=seed, components=components,
                                             series_id=sid)
        hd = fit_ds if history_dates is None else history_dates
        fb = cls(engine, fit, np.unique(hd), fit_ds, None)
        fb.series_ids = sid
        return fb, int(fg.T), out

    def spec(self) -> GridSpec:
        g = self.fit.grid
        return GridSpec(list(g.seasons), int(g.start_ns), int(g.t_scale_ns), g.t_change, g.holidays)

    def predict(self, ds_ns: np.ndarray, *, seed: int = 0, n_samples: int | None = None,
                components: bool = True, cap=None):
        """Forecast every series of the batch on the dates ``ds_ns`` (sorted).
        ``cap`` ([n, T] capacities on those dates) is required for logistic
        growth.  Returns (T, dict of float32 device tensors [n, T_pad])."""
        ds_ns = np.asarray(ds_ns, np.int64)
        fg = self.engine.predict_grid(self.fit, ds_ns)
        capd = None
        if self.engine.config.growth == "logistic":
            if cap is None:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            n = int(self.fit.theta.shape[0])
            capd = _dense(cap, n, fg.T, fg.T_pad, torch.device("cuda", self.engine.device))
        out = self.engine.predict(self.fit, fg, n_samples=n_samples, seed=seed,
                                  components=components, series_id=self.series_ids, cap=capd)
        return fg.T, out

    # -------------------------------------------------------- params store
    def to_record(self, keys: np.ndarray | None = None) -> dict:
        """Host arrays describing the fits (one params-store bucket): theta,
        scales, the grid spec (seasonalities, changepoints, holiday columns)
        and the model settings a forecast depends on (growth, seasonality
        mode, interval width), so a record is never served with a
        configuration it was not fitted under."""
        g = self.fit.grid
        cfg = self.engine.config
        rec = {
            "growth": np.str_(cfg.growth),
            "seasonality_mode": np.str_(cfg.seasonality_mode),
            "interval_width": np.float64(cfg.interval_width),
            "theta": self.fit.theta.cpu().numpy(),
            "y_scale": self.fit.y_scale.cpu().numpy(),
            "f": self.fit.f.cpu().numpy(),
            "status": self.fit.status.cpu().numpy(),
            "n_eval": self.fit.n_eval.cpu().numpy(),
            "t_change": g.t_change.cpu().numpy(),
            "start_ns": np.int64(g.start_ns),
            "t_scale_ns": np.int64(g.t_scale_ns),
            "history_dates": self.history_dates,
            "season_names": np.array([s[0] for s in g.seasons]),
            "season_periods": np.array([s[1] for s in g.seasons], dtype=np.float64),
            "season_orders": np.array([s[2] for s in g.seasons], dtype=np.int64),
        }
        rec.update(holiday_record(getattr(g, "holidays", None)))
        if keys is not None:
            rec["keys"] = np.asarray(keys, dtype=np.int64)
            if self.series_ids is None:
                rec["series_id"] = series_id(rec["keys"])
        if self.series_ids is not None:
            rec["series_id"] = self.series_ids.cpu().numpy()
        return rec

    @classmethod
    def from_record(cls, engine: E.Engine, rec: dict, rows=None) -> "FittedBatch":
        """Rebuild a (sub-)batch from a params-store record without refitting.
        Raises ValueError if the record was fitted under a growth /
        seasonality mode other than ``engine.config``'s or if theta's width
        does not match the record's grid (3 + S + K)."""
        check_record_config(rec, engine.config)
        dev = torch.device("cuda", engine.device)
        sel = slice(None) if rows is None else np.asarray(rows)
        theta = E._to_device_async(rec["theta"][sel], dev)
        n = theta.shape[0]
        seasons = [(str(a), float(b), int(c)) for a, b, c in
                   zip(rec["season_names"], rec["season_periods"], rec["season_orders"])]
        hol = holiday_from_record(rec)
        K = sum(2 * o for _, _, o in seasons) + (hol.n if hol is not None else 0)
        S = int(np.asarray(rec["t_change"]).shape[0])
        if theta.shape[1] != 3 + S + K:
            raise ValueError(f"record theta has {theta.shape[1]} columns; its grid needs "
                             f"3 + S + K = {3 + S + K}")
        spec = GridSpec(seasons, int(rec["start_ns"]), int(rec["t_scale_ns"]),
                        E._to_device_async(rec["t_change"], dev), hol)

        def _t(name, dtype):
            return E._to_device_async(rec[name][sel].astype(dtype), dev)

        fit = E.FitResult(spec, theta, _t("y_scale", np.float64), _t("f", np.float64),
                          _t("f", np.float64), _t("status", np.int32),
                          torch.zeros(n, dtype=torch.int32, device=dev), _t("n_eval", np.int32),
                          engine.config)
        sid = rec["series_id"][sel] if "series_id" in rec else None
        return cls(engine, fit, rec["history_dates"], None, sid)


class RaggedFittedBatch:
    """Series of several buckets (different date grids) fitted and forecast
    in single launches: one sub-grid per bucket, shared row stride, the
    kernels bind each workgroup to its series' grid (engine.RaggedGrid).
    Rows are the buckets' series in bucket order."""

    def __init__(self, engine: E.Engine, fit: E.FitResult, buckets, series_ids=None):
        self.engine = engine
        self.fit = fit
        self.buckets = list(buckets)
        sizes = [int(bk.Y.shape[0]) for bk in self.buckets]
        self.row0 = np.concatenate(([0], np.cumsum(sizes))).astype(np.int64)
        self.series_ids = None
        if series_ids is not None:
            self.series_ids = E._to_device_async(np.asarray(series_ids, dtype=np.int32),
                                                 fit.theta.device)

    @property
    def n(self) -> int:
        return int(self.fit.theta.shape[0])

    @classmethod
    def fit_buckets(cls, engine: E.Engine, buckets, series_ids=None, polish: bool | None = None,
                    cap=None) -> "RaggedFittedBatch":
        """Fit every series of ``buckets`` (each: fit_ds, history_dates, Y
        [n_b, T_b]) in one launch.  ``cap`` (logistic growth): a list with one
        [n_b, T_b] array per bucket."""
        cfg = engine.config
        dev = torch.device("cuda", engine.device)
        Tp = E.pad_rows(max(int(bk.fit_ds.shape[0]) for bk in buckets))
        starts, scales, seasons = [], [], None
        for bk in buckets:
            fds = np.asarray(bk.fit_ds, np.int64)
            if fds.shape[0] < 2:
                raise ValueError("Dataframe has less than 2 non-NaN rows.")
            start, t_scale = int(fds[0]), int(fds[-1] - fds[0])
            if t_scale <= 0:
                raise ValueError("history must span more than one distinct date")
            se = cfg.seasons(start, int(fds[-1]), min_positive_diff(fds))
            if seasons is not None and se != seasons:
                raise ValueError("ragged buckets must share their seasonalities (ragged_packs)")
            seasons = se
            starts.append(start)
            scales.append(t_scale)
        sizes = [int(bk.Y.shape[0]) for bk in buckets]
        rg = E.RaggedGrid.build([bk.fit_ds for bk in buckets], seasons, starts, scales,
                                np.repeat(np.arange(len(buckets)), sizes), device=engine.device,
                                T_pad=Tp, n_changepoints=cfg.n_changepoints,
                                changepoint_range=cfg.changepoint_range)
        n = int(sum(sizes))
        Yh = np.zeros((n, Tp), np.float64)
        caph = np.zeros((n, Tp), np.float64) if cfg.growth == "logistic" else None
        if cfg.growth == "logistic" and cap is None:
            raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
        r = 0
        for b, bk in enumerate(buckets):
            T = int(bk.fit_ds.shape[0])
            Yh[r:r + sizes[b], :T] = bk.Y
            if caph is not None:
                caph[r:r + sizes[b], :T] = cap[b]
            r += sizes[b]
        Yd = E._to_device_async(Yh, dev)
        capd = E._to_device_async(caph, dev) if caph is not None else None
        fit = engine.fit(rg, Yd, polish=polish, cap=capd)
        return cls(engine, fit, buckets, series_ids)

    def future(self, periods: int, freq="D", include_history: bool = True) -> list:
        """UPSTREAM make_future_dataframe per bucket (its own last date)."""
        return [future_dates(bk.history_dates, periods, freq, include_history=include_history)
                for bk in self.buckets]

    def predict(self, ds_list, *, seed: int = 0, n_samples: int | None = None,
                components: bool = True, cap=None):
        """Forecast every series on its bucket's dates (``ds_list[b]``, sorted)
        in one launch.  Returns (Tf per bucket, dict of float32 device tensors
        [n, T_pad]; row i valid up to its bucket's Tf).  ``cap`` (logistic):
        a list with one [n_b, Tf_b] array per bucket."""
        eng = self.engine
        fg = eng.predict_grid(self.fit, [np.asarray(d, np.int64) for d in ds_list])
        capd = None
        if eng.config.growth == "logistic":
            if cap is None:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            ch = np.zeros((self.n, fg.T_pad), np.float64)
            for b in range(len(self.buckets)):
                c = np.asarray(cap[b], np.float64)
                ch[self.row0[b]:self.row0[b + 1], :c.shape[1]] = c
            capd = E._to_device_async(ch, self.fit.theta.device)
        out = eng.predict(self.fit, fg, n_samples=n_samples, seed=seed, components=components,
                          series_id=self.series_ids, cap=capd)
        return [len(d) for d in ds_list], out

    def sub_batch(self, b: int) -> FittedBatch:
        """Bucket b's series as a plain FittedBatch on its own grid (the
        params-store unit; no copy of the fit beyond row views)."""
        sl = slice(int(self.row0[b]), int(self.row0[b + 1]))
        f = self.fit
        sub = E.FitResult(f.grid.grids[b], f.theta[sl], f.y_scale[sl], f.f[sl], f.f_stan[sl],
                          f.status[sl], f.n_iter[sl], f.n_eval[sl], f.config)
        bk = self.buckets[b]
        sid = self.series_ids[sl].cpu().numpy() if self.series_ids is not None else None
        return FittedBatch(self.engine, sub, bk.history_dates, bk.fit_ds, sid)
