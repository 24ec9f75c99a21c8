"""Ragged batches: series with different date grids (staggered launches,
different end dates) fitted and forecast in ONE launch per layout
(engine.RaggedGrid, pf_problem.grids / pf_predict_args.grids) instead of one
launch per distinct date set.  Reference: every applyInPandas group carries
its own history (notebooks/prophet/02_training.py:277-307).

Each workgroup binds its series' own grid, with the same rows per thread as a
batch of that grid alone, so the ragged path must reproduce the per-bucket
path bit for bit; it is also checked against the CPU oracle."""
import numpy as np
import pandas as pd
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import batch as B, synthetic, training
from distributed_forecasting_amd.engine import ProphetConfig
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

pytestmark = pytest.mark.gpu


def _buckets(n_stores=2, n_items=12, n_starts=4, n_ends=2, max_delay_days=500):
    df = synthetic.staggered_frame(n_stores, n_items, n_starts=n_starts, n_ends=n_ends,
                                   max_delay_days=max_delay_days)
    gkeys, rows = training.group_frame(df, ["store", "item"])
    ds_all = B.to_ns(df["ds"])
    y = df["y"].to_numpy(np.float64)
    bks = B.bucket_groups([ds_all[r] for r in rows], [y[r] for r in rows])
    return df, gkeys, bks


def test_ragged_fit_and_forecast_equal_per_bucket():
    """One ragged launch == one launch per bucket: theta, f, status, yhat and
    the Monte-Carlo intervals bit for bit (same series_id RNG streams)."""
    e = dfa.Engine(0, ProphetConfig.reference())
    df, gkeys, bks = _buckets()
    assert len(bks) >= 4
    packs = B.ragged_packs(bks, e.config)
    assert len(packs) == 1 and len(packs[0]) == len(bks)
    pkeys = np.concatenate([gkeys[bk.members] for bk in bks])
    rb = B.RaggedFittedBatch.fit_buckets(e, bks, series_ids=B.series_id(pkeys))
    futs = rb.future(90, "D")
    _, out = rb.predict(futs, seed=3)
    torch.cuda.synchronize()
    for j, bk in enumerate(bks):
        r0, r1 = int(rb.row0[j]), int(rb.row0[j + 1])
        fb = B.FittedBatch.fit_dense(e, bk.fit_ds, bk.Y, history_dates=bk.history_dates,
                                     series_ids=B.series_id(pkeys[r0:r1]))
        assert torch.equal(fb.fit.theta, rb.fit.theta[r0:r1]), j
        assert torch.equal(fb.fit.f, rb.fit.f[r0:r1])
        assert torch.equal(fb.fit.status, rb.fit.status[r0:r1])
        assert torch.equal(fb.fit.y_scale, rb.fit.y_scale[r0:r1])
        Tf, o1 = fb.predict(futs[j], seed=3)
        assert Tf == len(futs[j])
        for k in ("yhat", "yhat_lower", "yhat_upper", "trend", "trend_lower", "trend_upper",
                  "multiplicative_terms", "yearly", "weekly"):
            assert torch.equal(o1[k][:, :Tf], out[k][r0:r1, :Tf]), (j, k)
    assert np.all(rb.fit.status.cpu().numpy() == 70)


def test_ragged_sample_mode_equal_per_bucket():
    """interval_method='sample' (every row's 1000 samples; the history rows
    in k_predict_mc_hist, the horizon in k_predict_mc, both binding each
    series' own grid): one ragged launch == one launch per bucket, bit for
    bit, with and without trend bands."""
    cfg = ProphetConfig.reference()
    cfg.interval_method = "sample"
    e = dfa.Engine(0, cfg)
    df, gkeys, bks = _buckets()
    pkeys = np.concatenate([gkeys[bk.members] for bk in bks])
    rb = B.RaggedFittedBatch.fit_buckets(e, bks, series_ids=B.series_id(pkeys))
    futs = rb.future(90, "D")
    for comp in (False, True):
        _, out = rb.predict(futs, seed=5, components=comp)
        torch.cuda.synchronize()
        for j, bk in enumerate(bks):
            r0, r1 = int(rb.row0[j]), int(rb.row0[j + 1])
            fb = B.FittedBatch.fit_dense(e, bk.fit_ds, bk.Y, history_dates=bk.history_dates,
                                         series_ids=B.series_id(pkeys[r0:r1]))
            Tf, o1 = fb.predict(futs[j], seed=5, components=comp)
            keys = ("yhat", "yhat_lower", "yhat_upper") + (("trend_lower", "trend_upper") if comp else ())
            for k in keys:
                assert torch.equal(o1[k][:, :Tf], out[k][r0:r1, :Tf]), (comp, j, k)


def test_ragged_matches_oracle():
    """Per series on its own grid: objective <= oracle Stan + 1e-6 (rel),
    equal to the oracle's certified MAP within 1e-9, yhat within
    1e-6 y_scale of the oracle's point forecast at the MAP."""
    e = dfa.Engine(0, ProphetConfig.reference())
    df, gkeys, bks = _buckets(1, 8, n_starts=4, n_ends=2)
    rb = B.RaggedFittedBatch.fit_buckets(e, bks)
    futs = rb.future(90, "D")
    _, out = rb.predict(futs, seed=0)
    f = rb.fit.f.cpu().numpy()
    yh = out["yhat"].double().cpu().numpy()
    for j, bk in enumerate(bks):
        for i in range(bk.Y.shape[0]):
            s = int(rb.row0[j]) + i
            st = po.build_problem(bk.fit_ds, bk.Y[i])
            th_stan, f_stan, *_ = so.fit_setup(st)
            th, f_map, *_ = so.fit_map(st)
            assert f[s] <= f_stan + 1e-6 * abs(f_stan), (s, f[s], f_stan)
            assert abs(f[s] - f_map) <= 1e-9 * abs(f_map), (s, f[s], f_map)
            pt = po.predict_point(st, po.params_from_theta(th, st.problem.S), futs[j])
            d = np.abs(yh[s, :len(futs[j])] - pt["yhat"]).max() / st.hist.y_scale
            assert d <= 1e-6, (s, d)


def test_ragged_objective_gradient_and_hessian():
    """pf_objective_grad / pf_hessian on a ragged grid equal the per-grid calls."""
    e = dfa.Engine(0, ProphetConfig.reference())
    _, _, bks = _buckets(1, 10, n_starts=3, n_ends=2)
    rb = B.RaggedFittedBatch.fit_buckets(e, bks)
    rg = rb.fit.grid
    Tp = rg.T_pad
    n = rb.n
    Yd = torch.zeros((n, Tp), dtype=torch.float64, device="cuda")
    for j, bk in enumerate(bks):
        Yd[int(rb.row0[j]):int(rb.row0[j + 1]), :bk.fit_ds.shape[0]] = torch.from_numpy(bk.Y).cuda()
    ysc, ys, th0, _, _ = e.prepare(rg, Yd)
    th = rb.fit.theta
    f, g = e.objective_grad(rg, ys, th)
    H = e.hessian(rg, ys, th)
    for j, sg in enumerate(rg.grids):
        r0, r1 = int(rb.row0[j]), int(rb.row0[j + 1])
        ysc1, ys1, th01, _, _ = e.prepare(sg, Yd[r0:r1].contiguous())
        assert torch.equal(ysc1, ysc[r0:r1]) and torch.equal(th01, th0[r0:r1])
        f1, g1 = e.objective_grad(sg, ys1, th[r0:r1].contiguous())
        H1 = e.hessian(sg, ys1, th[r0:r1].contiguous())
        assert torch.equal(f1, f[r0:r1]) and torch.equal(g1, g[r0:r1]), j
        assert torch.equal(H1, H[r0:r1]), j


def test_forecast_store_items_staggered_matches_per_group():
    """The drop-in forecast_store_items on a staggered table (one ragged
    launch) returns the same rows as applyInPandas(forecast_store_item) run
    group by group: ds, keys, y by position, yhat (fp32) equal."""
    df = synthetic.staggered_frame(2, 6, n_starts=3, n_ends=2, max_delay_days=400)
    res = training.forecast_store_items(df)
    ref = []
    for (s, i), g in df.groupby(["store", "item"], sort=True):
        ref.append(training.forecast_store_item(g.reset_index(drop=True)))
    ref = pd.concat(ref, ignore_index=True)
    key = ["store", "item", "ds"]
    a = res.sort_values(key).reset_index(drop=True)
    b = ref.sort_values(key).reset_index(drop=True)
    assert len(a) == len(b)
    for c in ("store", "item", "ds"):
        assert np.array_equal(a[c].to_numpy(), b[c].to_numpy()), c
    assert np.array_equal(np.isnan(a["y"].to_numpy()), np.isnan(b["y"].to_numpy()))
    ya, yb = a["yhat"].to_numpy(np.float64), b["yhat"].to_numpy(np.float64)
    assert np.max(np.abs(ya - yb) / np.maximum(1.0, np.abs(yb))) <= 1e-5
    lo_a, hi_a = a["yhat_lower"].to_numpy(), a["yhat_upper"].to_numpy()
    assert np.all(lo_a <= ya + 1e-3) and np.all(hi_a >= ya - 1e-3)


def test_ragged_params_store_round_trip(tmp_path):
    """Each bucket of a ragged fit lands in the params store as its own
    record; the PyFunc model serves the same yhat."""
    from distributed_forecasting_amd import serving
    df = synthetic.staggered_frame(1, 6, n_starts=3, n_ends=1, max_delay_days=300)
    store = serving.ParamsStore(str(tmp_path / "ps"), ProphetConfig.reference())
    res = training.forecast_store_items(df, params_store=store)
    model = serving.ForecastStoreItemModel(store)
    fc = model.predict(None, res[["ds", "store", "item"]])
    m = res.merge(fc, on=["store", "item", "ds"], suffixes=("", "_srv"))
    assert len(m) > 0
    d = np.abs(m["yhat"].to_numpy(np.float64) - m["yhat_srv"].to_numpy(np.float64))
    assert np.max(d / np.maximum(1.0, np.abs(m["yhat"].to_numpy(np.float64)))) <= 1e-5


def test_ragged_irregular_grids_and_layout_split():
    """Series with NaN gaps (irregular date grids: dates read from the ds
    array, not generated) and a 20-day series (15 changepoints: its own pack)
    through forecast_store_items equal the per-group reference path."""
    df = synthetic.staggered_frame(1, 8, n_starts=3, n_ends=2, max_delay_days=300)
    y = df["y"].to_numpy().copy()
    g1 = np.flatnonzero((df["item"] == 2).to_numpy())
    y[g1[100:130]] = np.nan                       # a month missing
    g2 = np.flatnonzero((df["item"] == 5).to_numpy())
    y[g2[::97]] = np.nan                          # scattered NaNs
    df["y"] = y
    short = df[df["item"] == 7].tail(20).assign(item=9)
    df = pd.concat([df, short], ignore_index=True)
    gkeys, rows = training.group_frame(df, ["store", "item"])
    ds_all = B.to_ns(df["ds"])
    bks = B.bucket_groups([ds_all[r] for r in rows], [y_ for y_ in
                                                      (df["y"].to_numpy(np.float64)[r] for r in rows)])
    packs = B.ragged_packs(bks, ProphetConfig.reference())
    assert len(packs) == 2 and sorted(len(p) for p in packs)[0] == 1
    res = training.forecast_store_items(df)
    ref = pd.concat([training.forecast_store_item(g.reset_index(drop=True))
                     for _, g in df.groupby(["store", "item"], sort=True)], ignore_index=True)
    key = ["store", "item", "ds"]
    a = res.sort_values(key).reset_index(drop=True)
    b = ref.sort_values(key).reset_index(drop=True)
    assert len(a) == len(b)
    for c in key:
        assert np.array_equal(a[c].to_numpy(), b[c].to_numpy()), c
    ya, yb = a["yhat"].to_numpy(np.float64), b["yhat"].to_numpy(np.float64)
    assert np.max(np.abs(ya - yb) / np.maximum(1.0, np.abs(yb))) <= 1e-5


def test_ragged_never_takes_the_tile_path():
    """K3T needs one grid per tile: a ragged batch with tile_min_series=1 runs
    the per-series kernels and gives the same fits as the default."""
    e = dfa.Engine(0, ProphetConfig.reference())
    _, _, bks = _buckets(1, 20, n_starts=3, n_ends=1)
    rb = B.RaggedFittedBatch.fit_buckets(e, bks)
    rg = rb.fit.grid
    Yd = torch.zeros((rb.n, rg.T_pad), dtype=torch.float64, device="cuda")
    for j, bk in enumerate(bks):
        Yd[int(rb.row0[j]):int(rb.row0[j + 1]), :bk.fit_ds.shape[0]] = torch.from_numpy(bk.Y).cuda()
    f1 = e.fit(rg, Yd, tile_min_series=1)
    assert torch.equal(f1.theta, rb.fit.theta) and torch.equal(f1.status, rb.fit.status)
