"""Drop-in training / forecasting functions of the reference notebooks.

Reference (notebooks/prophet/02_training.py):
  train_model(history_pd, store=None) -> Prophet            :150-198
  make_prediction(model) -> DataFrame                        :201-205
  forecast_item(history_pd) -> DataFrame                     :208-223
  forecast_store_item(history_pd) -> DataFrame               :282-301
The per-group functions keep their signatures (Spark ``applyInPandas`` can
call them unchanged; each is a batch of one).  ``forecast_store_items`` is
the batched entry: it returns the rows that
``groupBy('store','item').applyInPandas(forecast_store_item, schema)`` would
(:305-307), computed bucket-by-bucket on the GPU.

Output assembly follows the reference exactly (row a9 of SURVEY.md §8):
``y`` is copied *by index position* from the incoming group frame (NaN past
its length), keys are broadcast from the group's first row, and the columns
are ``[ds, store, item, y, yhat, yhat_upper, yhat_lower]`` cast to the Spark
schema (keys int32, values float32, ds datetime64[ns] at midnight).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import batch as B
from . import engine as E
from .forecaster import SIMPLE_ATTRIBUTES, Prophet, get_engine

HORIZON_DAYS = 90
SCHEMA_STORE_ITEM = ["ds", "store", "item", "y", "yhat", "yhat_upper", "yhat_lower"]
SCHEMA_ITEM = ["ds", "item", "y", "yhat", "yhat_upper", "yhat_lower"]


def reference_model(**over) -> Prophet:
    """The constructor call of 02_training.py:162-169."""
    kw = dict(interval_width=0.95, growth="linear", daily_seasonality=False,
              weekly_seasonality=True, yearly_seasonality=True,
              seasonality_mode="multiplicative")
    kw.update(over)
    return Prophet(**kw)


def extract_params(pr_model: Prophet) -> dict:
    """02_training.py:146-147 (serialize.SIMPLE_ATTRIBUTES)."""
    return {attr: getattr(pr_model, attr) for attr in SIMPLE_ATTRIBUTES}


# ---------------------------------------------------------------------------
# per-group API (batch of one)
# ---------------------------------------------------------------------------
def train_model(history_pd: pd.DataFrame, store: int = None, *, params_store=None,
                cv_metrics: bool = False, device=None) -> Prophet:
    """02_training.py:150-198 without MLflow: fit the reference model.

    ``params_store`` (a ``ParamsStore``) receives the fitted parameters (the
    reference logs params + model artifact to MLflow, :190-196).  With
    ``cv_metrics`` the reference's cross-validation metrics (:178-188) are
    computed and attached as ``model.metrics``."""
    model = reference_model(device=device)
    model.fit(history_pd)
    item = history_pd["item"].iloc[0]
    model.run_name = f"run_item_{item}_store_{store if store else 'all'}"
    if cv_metrics:
        from .diagnostics import cv_metrics_batch
        fds = B.to_ns(model.history["ds"])
        y = model.history["y"].to_numpy(np.float64)
        model.metrics = {k: float(v[0]) for k, v in
                         cv_metrics_batch(model._batch.engine, fds, y[None, :]).items()}
    if params_store is not None:
        key = (int(store) if store else -1, int(item))
        params_store.put_batch(model._batch, np.array([key], dtype=np.int64))
    return model


def make_prediction(model: Prophet) -> pd.DataFrame:
    """02_training.py:201-205."""
    future_pd = model.make_future_dataframe(periods=HORIZON_DAYS, freq="d",
                                            include_history=True)
    return model.predict(future_pd)


def _assemble_one(history_pd, forecast_pd, key_cols):
    out = pd.DataFrame({"ds": forecast_pd["ds"].values})
    yin = history_pd["y"].to_numpy(np.float64)
    y = np.full(len(out), np.nan)
    m = min(len(out), len(yin))
    y[:m] = yin[:m]                       # forecast_pd['y'] = history_pd['y'] (by position)
    for k in key_cols:
        out[k] = np.int32(history_pd[k].iloc[0])
    out["y"] = y.astype(np.float32)
    for k in ("yhat", "yhat_upper", "yhat_lower"):
        out[k] = forecast_pd[k].to_numpy(np.float32)
    return out


def forecast_item(history_pd: pd.DataFrame) -> pd.DataFrame:
    """02_training.py:208-223 (item-level, schema of :233)."""
    model = train_model(history_pd)
    forecast_pd = make_prediction(model)
    return _assemble_one(history_pd.reset_index(drop=True), forecast_pd, ["item"])[SCHEMA_ITEM]


def forecast_store_item(history_pd: pd.DataFrame) -> pd.DataFrame:
    """02_training.py:282-301 (schema of :307)."""
    store = history_pd["store"].iloc[0]
    model = train_model(history_pd, store=store)
    forecast_pd = make_prediction(model)
    return _assemble_one(history_pd.reset_index(drop=True), forecast_pd,
                         ["store", "item"])[SCHEMA_STORE_ITEM]


# ---------------------------------------------------------------------------
# batched API
# ---------------------------------------------------------------------------
def group_frame(df: pd.DataFrame, keys):
    """Split a long frame into groups (original row order kept inside each
    group, like the frames applyInPandas hands to the UDF).
    Returns (group keys [G, k] int64, list of row-position arrays)."""
    cols = [df[k].to_numpy(np.int64) for k in keys]
    n = cols[0].shape[0] if cols else 0
    if n == 0:
        return np.zeros((0, len(keys)), np.int64), []
    # one sortable code per row when the keys fit (store / item ids): a
    # frame already grouped (the usual layout of the sales table) needs no
    # sort at all; otherwise one stable argsort of the codes
    lo = [int(c.min()) for c in cols]
    span = [int(c.max()) - l + 1 for c, l in zip(cols, lo)]
    if float(np.prod(np.asarray(span, np.float64))) < 2.0 ** 62:
        code = cols[0] - lo[0]
        for c, l, sp in zip(cols[1:], lo[1:], span[1:]):
            code = code * sp + (c - l)
        if bool(np.all(code[1:] >= code[:-1])):
            order, sc = np.arange(n), code
        else:
            order = np.argsort(code, kind="stable")
            sc = code[order]
        brk = np.flatnonzero(sc[1:] != sc[:-1]) + 1
    else:
        kv = np.stack(cols, axis=1)
        order = np.lexsort(kv.T[::-1])              # stable: keeps row order in a group
        sk = kv[order]
        brk = np.flatnonzero(np.any(sk[1:] != sk[:-1], axis=1)) + 1
    starts = np.concatenate(([0], brk))
    ends = np.concatenate((brk, [n]))
    first = order[starts]
    return np.stack([c[first] for c in cols], axis=1), [order[s:e] for s, e in zip(starts, ends)]


def dense_guess(df: pd.DataFrame, keys, value: str | None = "y"):
    """The O(groups + dates) half of ``dense_frame``: reads the layout off the
    first group (its length T = the first key change) and checks what that
    costs nothing to check (T divides the rows, strictly increasing dates in
    the first group, strictly increasing group keys at every T-th row).
    Returns (group keys [n, k] int64, dates [T] int64 ns, values [n, T]
    float64 view or None, verify) or None; ``verify`` (a RowChecks: start()
    submits, verify() waits) runs the O(rows) checks (every group on the first group's dates, keys constant inside each
    group, no NaN value) and must return True before the guess is used for
    anything a caller can observe.  Callers launch the GPU work on the guess
    and verify while it runs."""
    N = len(df)
    if N == 0 or (value is not None and value not in df):
        return None
    cols = [df[k].to_numpy() for k in keys]
    if any(c.dtype.kind not in "iu" for c in cols):
        return None
    # first key change: scan growing prefixes (a sorted table finds it in
    # the first chunk)
    T, m = N, 4096
    while True:
        lim = min(N, m)
        ch = np.zeros(lim - 1, bool)
        for c in cols:
            ch |= c[1:lim] != c[0]
        hit = np.flatnonzero(ch)
        if hit.shape[0]:
            T = int(hit[0]) + 1
            break
        if lim == N:
            break
        m *= 8
    n = N // T
    if T < 2 or n * T != N:
        return None
    gkeys = np.stack([c[::T].astype(np.int64) for c in cols], axis=1)
    if n > 1:
        # strictly increasing keys (lexicographic): the general path's group
        # order, and no key split over two runs
        inc = np.zeros(n - 1, bool)
        eq = np.ones(n - 1, bool)
        for j in range(len(keys)):
            a = gkeys[:, j]
            inc |= eq & (a[1:] > a[:-1])
            eq &= a[1:] == a[:-1]
        if not bool(inc.all()):
            return None
    ds = df["ds"].to_numpy()
    if ds.dtype.kind != "M":
        return None
    if ds.dtype != np.dtype("datetime64[ns]"):
        ds = ds.astype("datetime64[ns]")
    dsi = ds.view(np.int64).reshape(n, T)
    ds0 = np.array(dsi[0])
    if not bool(np.all(ds0[1:] > ds0[:-1])):
        return None
    Y = df[value].to_numpy(np.float64).reshape(n, T) if value is not None else None

    def rows_ok(a: int, b: int) -> bool:
        for c in cols:
            c2 = c.reshape(n, T)[a:b]
            if not np.array_equal(c2.min(axis=1), c2.max(axis=1)):
                return False
        if not bool((dsi[max(a, 1):b] == ds0).all()):
            return False
        return Y is None or not bool(np.isnan(Y[a:b]).any())
    return gkeys, ds0, Y, RowChecks(rows_ok, n)


class RowChecks:
    """The O(rows) half of a layout check, run over group ranges on a small
    thread pool (numpy releases the GIL in its loops): ``start()`` submits
    the ranges and returns at once, so the checks overlap the caller's GPU
    launches and output assembly; calling the object waits and returns True
    when every range passed."""
    _pool = None
    CHUNKS = 4

    def __init__(self, fn, n: int):
        self.fn, self.n, self.futs = fn, n, None

    @classmethod
    def pool(cls):
        if cls._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            cls._pool = ThreadPoolExecutor(max_workers=cls.CHUNKS, thread_name_prefix="pf-rowcheck")
        return cls._pool

    def start(self) -> "RowChecks":
        if self.futs is None:
            k = min(self.CHUNKS, self.n)
            cut = [self.n * i // k for i in range(k + 1)]
            self.futs = [self.pool().submit(self.fn, a, b) for a, b in zip(cut[:-1], cut[1:])]
        return self

    def __call__(self) -> bool:
        self.start()
        return all(f.result() for f in self.futs)


def dense_frame(df: pd.DataFrame, keys, value: str | None = "y"):
    """The sales table's usual layout without per-group work: the frame is
    grouped, its groups come in increasing key order, every group holds the
    same strictly increasing dates and no ``value`` is NaN.  Returns (group
    keys [n, k] int64, dates [T] int64 ns, values [n, T] float64 — a view of
    the ``value`` column, None if ``value`` is None) or None when any of that
    does not hold (then ``group_frame`` + ``bucket_groups`` run).  Vectorised
    checks only: O(rows) with no Python loop over groups."""
    g = dense_guess(df, keys, value)
    if g is None or not g[3]():
        return None
    return g[:3]


def _empty_frame(cols, keys):
    return pd.DataFrame({c: pd.Series(dtype=("datetime64[ns]" if c == "ds" else
                                             np.int32 if c in keys else np.float32))
                         for c in cols})


def forecast_store_items(df: pd.DataFrame, keys=("store", "item"), *, periods: int = HORIZON_DAYS,
                         freq="d", config: E.ProphetConfig | None = None, device=None,
                         seed: int = 0, params_store=None, rank: int = 0,
                         world_size: int = 1, return_fits: bool = False,
                         cv_metrics: bool = False, return_metrics: bool = False,
                         _guess: bool = True):
    """Batched equivalent of
    ``df.groupBy(*keys).applyInPandas(forecast_store_item, schema)``.

    With ``world_size > 1`` only the groups whose splitmix64 key hash maps to
    ``rank`` are processed; ``parallel.gather_frames``
    collects the per-rank frames.

    ``cv_metrics``: the reference's ``train_model`` cross-validation
    (02_training.py:178-188: horizon 90 days, period 360, initial 730, then
    ``performance_metrics``) for every series, per bucket on the GPU (fold
    refits + fold forecasts + K6).  The per-series metrics (the means over
    horizons of mse, rmse, mae, mape, ... — what :187-192 logs to MLflow) go
    into each params-store record and, with ``return_metrics``, into a
    DataFrame [keys..., *CV_METRICS].

    Returns the forecast frame; with ``return_fits`` / ``return_metrics`` a
    tuple (frame, fits, metrics) holding the requested extras in that order."""
    from . import diagnostics
    from . import _lib as L
    keys = list(keys)
    cfg = config or E.ProphetConfig.reference()
    eng = get_engine(cfg, device)
    dev = torch.device("cuda", eng.device)
    cols = ["ds"] + keys + ["y", "yhat", "yhat_upper", "yhat_lower"]
    # the sorted sales table: one bucket, no per-group Python.  The layout is
    # read off the first group and the O(rows) checks run while the GPU works
    # (dense_guess); a frame that fails them is redone by the general path
    dense = dense_guess(df, keys) if _guess else None
    verify = None
    if dense is not None:
        gkeys, ds0, Y, verify = dense
        if world_size > 1:
            mine = np.flatnonzero(B.shard_of(gkeys, world_size) == rank)
            gkeys, Y = gkeys[mine], Y[mine]
        buckets = [B.Bucket(ds0, ds0, Y, np.arange(gkeys.shape[0]))] if gkeys.shape[0] else []
        y_list = None
    else:
        gkeys, rows = group_frame(df, keys)
        if world_size > 1:
            mine = np.flatnonzero(B.shard_of(gkeys, world_size) == rank)
            gkeys = gkeys[mine]
            rows = [rows[i] for i in mine]
        ds_all = B.to_ns(df["ds"])
        y_all = df["y"].to_numpy(np.float64)
        ds_list = [ds_all[r] for r in rows]
        y_list = [y_all[r] for r in rows]
        buckets = B.bucket_groups(ds_list, y_list)

    # phase 1: every launch (fit, forecast, CV folds) and the asynchronous
    # D2H of each forecast block into pinned memory, so the host assembles
    # the output columns below while the GPU works
    launched = []
    for pack in B.ragged_packs(buckets, cfg):
        bks = [buckets[b] for b in pack]
        if len(pack) == 1:
            bk = bks[0]
            bkeys = gkeys[bk.members]
            futs = [B.future_dates(bk.history_dates, periods, freq, include_history=True)]
            if cv_metrics or cfg.growth == "logistic":
                Yd = B._dense(bk.Y, bk.Y.shape[0], bk.Y.shape[1], bk.Y.shape[1], dev) \
                    if cv_metrics else bk.Y
                fb = B.FittedBatch.fit_dense(eng, bk.fit_ds, Yd, history_dates=bk.history_dates,
                                             series_ids=B.series_id(bkeys))
                Tf, out = fb.predict(futs[0], seed=seed, components=False)
            else:
                # fit + forecast in one launch (pf_fit_forecast)
                Yd = bk.Y
                fb, Tf, out = B.FittedBatch.fit_forecast_dense(
                    eng, bk.fit_ds, bk.Y, futs[0], history_dates=bk.history_dates,
                    series_ids=B.series_id(bkeys), seed=seed, components=False)
            blk = torch.stack([out[k][:, :Tf] for k in ("yhat", "yhat_upper", "yhat_lower")])
            row0 = [0, len(bk.members)]
            subs = [(bkeys, fb, Yd)]
        else:
            pkeys = np.concatenate([gkeys[bk.members] for bk in bks])
            rb = B.RaggedFittedBatch.fit_buckets(eng, bks, series_ids=B.series_id(pkeys))
            futs = rb.future(periods, freq)
            _, out = rb.predict(futs, seed=seed, components=False)
            blk = torch.stack([out[k] for k in ("yhat", "yhat_upper", "yhat_lower")])
            row0 = [int(v) for v in rb.row0]
            subs = [(pkeys[row0[j]:row0[j + 1]], rb.sub_batch(j), bk.Y) for j, bk in enumerate(bks)]
        host = torch.empty(blk.shape, dtype=blk.dtype, pin_memory=True)
        host.copy_(blk, non_blocking=True)
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(dev))
        mets = []
        if cv_metrics:
            for (bkeys, fb, Yc), bk in zip(subs, bks):
                mets.append(diagnostics.cv_metrics_device(
                    eng, bk.fit_ds, Yc, seasons=fb.fit.grid.seasons,
                    series_ids=B.series_id(bkeys), seed=seed))
        launched.append((bks, futs, row0, host, done, subs, mets))

    if verify is not None:
        # started after the launches: the row checks would otherwise compete
        # with the pinned staging copy of Y for memory bandwidth
        verify.start()
    if verify is not None and not verify():
        # not the dense layout after all: the launches above are dropped
        # (nothing was stored) and the general path runs
        return forecast_store_items(df, keys, periods=periods, freq=freq, config=config,
                                    device=device, seed=seed, params_store=params_store,
                                    rank=rank, world_size=world_size, return_fits=return_fits,
                                    cv_metrics=cv_metrics, return_metrics=return_metrics,
                                    _guess=False)

    # phase 2: output columns (schema of 02_training.py:307); y is copied by
    # position from each group's frame (NaN past its rows)
    frames = []
    for bks, futs, row0, host, done, subs, mets in launched:
        for j, bk in enumerate(bks):
            fut = futs[j]
            Tf = len(fut)
            n = len(bk.members)
            bkeys = gkeys[bk.members]
            fr = {"ds": np.tile(fut.view("datetime64[ns]"), n)}
            for c, k in enumerate(keys):
                fr[k] = np.repeat(bkeys[:, c].astype(np.int32), Tf)
            yin = np.empty((n, Tf), np.float32)
            if y_list is None:
                T = bk.Y.shape[1]
                m = min(T, Tf)
                yin[:, :m] = bk.Y[:, :m]
                yin[:, m:] = np.nan
            else:
                yin[:] = np.nan
                for i, g in enumerate(bk.members):
                    v = y_list[g]
                    m = min(Tf, len(v))
                    yin[i, :m] = v[:m]
            fr["y"] = yin.reshape(-1)
            frames.append((fr, host, done, row0[j], row0[j + 1], Tf))
    outs = []
    for fr, host, done, r0, r1, Tf in frames:
        done.synchronize()
        h = host.numpy()
        for c, k in enumerate(("yhat", "yhat_upper", "yhat_lower")):
            v = h[c, r0:r1, :Tf]
            fr[k] = v.reshape(-1) if v.flags.c_contiguous else np.ascontiguousarray(v).reshape(-1)
        outs.append(fr)

    # phase 3: params store records (with the CV metrics), extras
    fits, met_frames = [], []
    for bks, futs, row0, host, done, subs, mets in launched:
        for j, (bkeys, fb, _) in enumerate(subs):
            mh = mets[j].cpu().numpy() if mets else None
            if params_store is not None:
                params_store.put_batch(fb, bkeys, metrics=mh)
            if return_fits:
                fits.append((bkeys, fb))
            if mh is not None:
                mf = {k: bkeys[:, c].astype(np.int32) for c, k in enumerate(keys)}
                mf.update({name: mh[:, c] for c, name in enumerate(L.CV_METRICS)})
                met_frames.append(pd.DataFrame(mf))
    if outs:
        res = pd.DataFrame({c: (outs[0][c] if len(outs) == 1 else
                                np.concatenate([f[c] for f in outs])) for c in cols}, copy=False)
    else:
        res = _empty_frame(cols, keys)
    if not (return_fits or return_metrics):
        return res
    extra = [res]
    if return_fits:
        extra.append(fits)
    if return_metrics:
        if not cv_metrics:
            raise ValueError("return_metrics needs cv_metrics=True")
        extra.append(pd.concat(met_frames, ignore_index=True) if met_frames else
                     pd.DataFrame({**{k: pd.Series(dtype=np.int32) for k in keys},
                                   **{m: pd.Series(dtype=np.float64) for m in L.CV_METRICS}}))
    return tuple(extra)


def forecast_items(df: pd.DataFrame, **kw):
    """Batched ``groupBy('item').applyInPandas(forecast_item, ...)`` (:232-233)."""
    return forecast_store_items(df, keys=("item",), **kw)


def allocate_forecasts(item_forecast: pd.DataFrame, sales: pd.DataFrame,
                       training_date=None) -> pd.DataFrame:
    """The item-level stage's allocation (02_training.py:235-247): store
    ratios ``sales / SUM(sales) OVER (PARTITION BY item)`` over the raw
    (store, item, sales) table, joined on item; ``y`` and ``yhat`` scaled by
    the ratio.  Columns ``date, store, item, sales, forecast, training_date``
    — the ``allocated_forecasts`` table the fine-grained stage reads back
    (with NaN ``sales`` on the 90 future rows)."""
    val = "sales" if "sales" in sales else "y"
    tot = sales.groupby(["store", "item"], as_index=False)[val].sum()
    tot["ratio"] = tot[val] / tot.groupby("item")[val].transform("sum")
    res = item_forecast.merge(tot[["store", "item", "ratio"]], on="item")
    out = pd.DataFrame({
        "date": res["ds"],
        "store": res["store"].astype(np.int32),
        "item": res["item"].astype(np.int32),
        "sales": (res["y"] * res["ratio"]).astype(np.float32),
        "forecast": (res["yhat"] * res["ratio"]).astype(np.float32),
    })
    out["training_date"] = pd.Timestamp.today().normalize() if training_date is None else training_date
    return out


def forecast_partitions(keys=("store", "item"), **kw):
    """A ``mapInPandas``-compatible function: every group frame of a Spark
    partition (an iterator of pandas frames holding whole groups, e.g. after
    ``repartition('store', 'item')``) goes to the GPU in one batched call
    instead of one Python call per group; yields the same rows and schema as
    ``applyInPandas(forecast_store_item, ...)``."""
    def run(frames):
        parts = [f for f in frames if len(f)]
        if parts:
            yield forecast_store_items(pd.concat(parts, ignore_index=True), keys=keys, **kw)
    return run
