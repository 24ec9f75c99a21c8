"""Batched cross-validation metrics.

Reference: ``train_model`` runs ``cross_validation(model, horizon='90 days',
period='360 days', initial='730 days')`` then ``performance_metrics`` and logs
``{k: cv_metrics[k].mean() for k in ['mse', 'mae', 'mape']}``
(notebooks/prophet/02_training.py:178-188).

Here every fold of every series in a bucket is one extra batched fit on the
fold's own grid (UPSTREAM prophet_copy: same seasonalities, changepoints
re-placed on the truncated history), the fold forecasts stay on the device,
and K6 (``pf_cv_metrics``) reduces them to per-series metrics.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L
from . import batch as B
from . import engine as E

NS_PER_DAY = E.NS_PER_DAY


def generate_cutoffs(ds_ns, horizon_ns: int, initial_ns: int, period_ns: int) -> list:
    """UPSTREAM diagnostics.generate_cutoffs (host date arithmetic)."""
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
                cutoff = int(ds_ns[ds_ns <= cutoff].max()) - horizon_ns
        result.append(cutoff)
    result = result[:-1]
    if len(result) == 0:
        raise ValueError("Less data than horizon after initial window. "
                         "Make horizon or initial shorter.")
    return list(reversed(result))


def cv_metrics_device(engine: E.Engine, fit_ds: np.ndarray, Y, *, horizon_days: float = 90,
                      period_days: float = 360, initial_days: float = 730,
                      rolling_window: float = 0.1, seasons=None, coverage: bool = False,
                      seed: int = 0, series_ids=None, priors=None,
                      packed: bool | None = None) -> torch.Tensor:
    """[n, 7] float64 device tensor: mse, rmse, mae, mape, smape, coverage,
    mdape (each the mean over horizons of the rolled metric) for every row of
    Y.  ``packed``: None picks the launch shape (every fold in one ragged
    launch while the batch is below the tiled path's size, else one launch
    per fold); True / False force it (the two are bitwise equal)."""
    fit_ds = np.asarray(fit_ds, np.int64)
    dev = torch.device("cuda", engine.device)
    Yt = Y if isinstance(Y, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(Y, np.float64))
    Yt = Yt.to(dev, torch.float64)
    n = Yt.shape[0]
    horizon = int(round(horizon_days * NS_PER_DAY))
    cutoffs = generate_cutoffs(fit_ds, horizon, int(round(initial_days * NS_PER_DAY)),
                               int(round(period_days * NS_PER_DAY)))
    if seasons is None:
        seasons = engine.config.seasons(int(fit_ds[0]), int(fit_ds[-1]),
                                        B.min_positive_diff(fit_ds))
    y_parts, f_parts, lo_parts, hi_parts, h_parts = [], [], [], [], []
    folds = []
    for c in cutoffs:
        tr = fit_ds <= c
        if int(tr.sum()) < 2:
            raise ValueError("Less than two datapoints before cutoff. Increase initial window.")
        folds.append((c, int(tr.sum()), np.flatnonzero((fit_ds > c) & (fit_ds <= c + horizon))))
    sids = None
    if series_ids is not None:
        sids = torch.from_numpy(np.ascontiguousarray(series_ids, dtype=np.int32)).to(dev)
    can_pack = priors is None and len(folds) > 1 and engine.config.growth != "logistic"
    if packed is None:
        packed = can_pack and n * len(folds) < engine.fit_opts().tile_min_series
    elif packed and not can_pack:
        raise ValueError("packed folds need shared priors, >1 fold and non-logistic growth")
    if packed:
        # every fold's refit and forecast in ONE launch per kernel: the folds
        # are the sub-grids of a ragged batch (same seasonalities, each with
        # its own changepoints on its truncated history, UPSTREAM
        # prophet_copy), bitwise the per-fold launches (tests/test_gpu_ragged.py)
        # while the folds' slow series overlap instead of each launch
        # waiting for its own slowest series
        cfg = engine.config
        Tp = E.pad_rows(max(k for _, k, _ in folds))
        G = len(folds)
        rg = E.RaggedGrid.build([fit_ds[:k] for _, k, _ in folds], seasons,
                                [int(fit_ds[0])] * G, [int(fit_ds[k - 1] - fit_ds[0]) for _, k, _ in folds],
                                np.repeat(np.arange(G), n), device=engine.device, T_pad=Tp,
                                n_changepoints=cfg.n_changepoints,
                                changepoint_range=cfg.changepoint_range)
        Yp = torch.zeros((G * n, Tp), dtype=torch.float64, device=dev)
        for g, (_, k, _) in enumerate(folds):
            Yp[g * n:(g + 1) * n, :k] = Yt[:, :k]
        fit = engine.fit(rg, Yp)
        fg = engine.predict_grid(fit, [fit_ds[te] for _, _, te in folds])
        out = engine.predict(fit, fg, n_samples=None if coverage else 0, seed=seed,
                             components=False,
                             series_id=sids.repeat(G) if sids is not None else None)
        for g, (c, k, te) in enumerate(folds):
            Tf = len(te)
            y_parts.append(Yt[:, te[0]:te[-1] + 1] if np.all(np.diff(te) == 1) else Yt[:, te])
            f_parts.append(out["yhat"][g * n:(g + 1) * n, :Tf])
            lo_parts.append(out["yhat_lower"][g * n:(g + 1) * n, :Tf])
            hi_parts.append(out["yhat_upper"][g * n:(g + 1) * n, :Tf])
            h_parts.append(fit_ds[te] - c)
        cutoffs = []
    for c in cutoffs:
        tr = fit_ds <= c
        if int(tr.sum()) < 2:
            raise ValueError("Less than two datapoints before cutoff. Increase initial window.")
        te = np.flatnonzero((fit_ds > c) & (fit_ds <= c + horizon))
        Ttr = int(tr.sum())
        fb = B.FittedBatch.fit_dense(engine, fit_ds[:Ttr], Yt[:, :Ttr], series_ids=series_ids,
                                     seasons=seasons, priors=priors)
        Tf, out = fb.predict(fit_ds[te], seed=seed,
                             n_samples=None if coverage else 0, components=False)
        y_parts.append(Yt[:, te[0]:te[-1] + 1] if np.all(np.diff(te) == 1) else Yt[:, te])
        f_parts.append(out["yhat"][:, :Tf])
        lo_parts.append(out["yhat_lower"][:, :Tf])
        hi_parts.append(out["yhat_upper"][:, :Tf])
        h_parts.append(fit_ds[te] - c)
    h = np.concatenate(h_parts)
    order = np.argsort(h, kind="stable")
    hs = h[order]
    brk = np.flatnonzero(hs[1:] != hs[:-1]) + 1
    gstart = np.concatenate(([0], brk, [len(hs)])).astype(np.int32)
    M = len(hs)
    w = min(max(int(rolling_window * M), 1), M)
    perm = torch.from_numpy(order).to(dev)
    yy = torch.cat(y_parts, 1)[:, perm].contiguous()
    ff = torch.cat(f_parts, 1)[:, perm].contiguous()
    lo = torch.cat(lo_parts, 1)[:, perm].contiguous() if coverage else None
    hi = torch.cat(hi_parts, 1)[:, perm].contiguous() if coverage else None
    gs = torch.from_numpy(gstart).to(dev)
    met = torch.empty((n, len(L.CV_METRICS)), dtype=torch.float64, device=dev)
    a = L.PfCvArgs(n, M, len(gstart) - 1, w, gs.data_ptr(), yy.data_ptr(), ff.data_ptr(),
                   lo.data_ptr() if lo is not None else None,
                   hi.data_ptr() if hi is not None else None, met.data_ptr())
    rc = engine.ctx.lib.pf_cv_metrics(engine.ctx.h, ctypes.byref(a),
                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    engine.ctx.check(rc, "pf_cv_metrics")
    met._keep = (yy, ff, lo, hi, gs)
    return met


def cv_metrics_batch(engine: E.Engine, fit_ds, Y, **kw) -> dict:
    """Host dict metric -> [n] numpy array (NaN where UPSTREAM skips)."""
    met = cv_metrics_device(engine, fit_ds, Y, **kw).cpu().numpy()
    return {name: met[:, i] for i, name in enumerate(L.CV_METRICS)}


def insample_metrics(engine: E.Engine, y: torch.Tensor, yhat: torch.Tensor,
                     yhat_lower: torch.Tensor | None = None,
                     yhat_upper: torch.Tensor | None = None, mdape: bool = True) -> torch.Tensor:
    """[n, 7] float64 device tensor of K6's metric set over the history rows
    (one horizon group, window = every row: the plain means, the median for
    MDAPE; MAPE NaN where UPSTREAM skips it).  ``y`` [n, T] float64 and
    ``yhat`` [n, >= T] float32 on the device; the per-series validation
    metrics the multi-GPU path all-gathers (the reference logs its CV
    metrics per series to MLflow, 02_training.py:187-192).  ``mdape=False``
    skips the median (NaN): the reference logs mse / mae / mape only."""
    met, a = insample_args(y, yhat, yhat_lower, yhat_upper, mdape)
    rc = engine.ctx.lib.pf_cv_metrics(engine.ctx.h, ctypes.byref(a),
                                      ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream))
    engine.ctx.check(rc, "pf_cv_metrics")
    return met


def insample_args(y: torch.Tensor, yhat: torch.Tensor, yhat_lower: torch.Tensor | None = None,
                  yhat_upper: torch.Tensor | None = None, mdape: bool = True):
    """The [n, 7] output tensor and the pf_cv_args of ``insample_metrics``
    (also handed to pf_fit_forecast).  The tensors the args point at are
    kept alive by both (``met._keep``, ``args._keep``)."""
    n, T = int(y.shape[0]), int(y.shape[1])
    dev = y.device

    def rows(t):
        # read in place (row stride ld) when the rows are unit-stride: no copy
        # kernels in the step (the padded history / forecast buffers)
        if t is None:
            return None, 0
        t = t[:, :T]
        if t.stride(1) != 1 or t.stride(0) < T:
            t = t.contiguous()
        return t, int(t.stride(0))
    yy, ld_y = rows(y)
    ff, ld_f = rows(yhat)
    lo, ld_lo = rows(yhat_lower)
    hi, ld_hi = rows(yhat_upper)
    if lo is not None and (ld_lo != ld_f or ld_hi != ld_f):
        ff, lo, hi = ff.contiguous(), lo.contiguous(), hi.contiguous()
        ld_f = T
    met = torch.empty((n, len(L.CV_METRICS)), dtype=torch.float64, device=dev)
    # group_start NULL: one horizon group of every row (window = T)
    a = L.PfCvArgs(n, T, 1, T, None, yy.data_ptr(), ff.data_ptr(),
                   lo.data_ptr() if lo is not None else None,
                   hi.data_ptr() if hi is not None else None, met.data_ptr(), ld_y, ld_f,
                   0 if mdape else 1)
    met._keep = (yy, ff, lo, hi)
    a._keep = met._keep
    return met, a
