"""GPU parity of the tiled fit kernel K3T (16 series per workgroup, FP64 MFMA
row pass X[T x K].B[K x 16] and X'[K x T].W[T x 16], per-series lane-quad
Stan L-BFGS) against the per-series kernel K3 and the CPU oracle.  The tile
path is forced with tile_min_series=1 on small batches; large batches take
it by default (pf_fit_opts.tile_min_series = 2048)."""
import numpy as np
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
from distributed_forecasting_amd.engine import ProphetConfig
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

pytestmark = pytest.mark.gpu


def _setup(n, mode="multiplicative", growth="linear", ds=None, config_index=2):
    c = ProphetConfig.reference()
    c.seasonality_mode = mode
    c.growth = growth
    e = dfa.Engine(0, c)
    ds = synthetic.daily_dates() if ds is None else ds
    seasons = c.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    Y = synthetic.sales_matrix(n, ds, config_index=config_index)
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    return e, g, ds, Y, Yd


@pytest.mark.parametrize("mode", ["multiplicative", "additive"])
def test_tile_reaches_same_certified_map(mode):
    """37 series (two full tiles + a ragged tail tile, one constant series):
    tile pass 0 + polish reaches the per-series path's certified MAP."""
    e, g, ds, Y, Yd = _setup(37, mode)
    Yd[5, :g.T] = 7.0                                   # constant series
    ft = e.fit(g, Yd, tile_min_series=1)
    fs = e.fit(g, Yd, tile_min_series=-1)
    st_t, st_s = ft.status.cpu().numpy(), fs.status.cpu().numpy()
    assert st_t[5] == 50 and st_s[5] == 50
    ok = np.arange(37) != 5
    assert np.all(st_t[ok] == 70) and np.all(st_s[ok] == 70), (st_t, st_s)
    f_t, f_s = ft.f.cpu().numpy()[ok], fs.f.cpu().numpy()[ok]
    assert np.all(np.abs(f_t - f_s) <= 1e-9 * np.abs(f_s)), np.max(np.abs(f_t - f_s) / np.abs(f_s))
    assert np.array_equal(ft.theta[5].cpu().numpy(), fs.theta[5].cpu().numpy())


def test_tile_stan_phase_matches_oracle():
    """fit_mode='stan' through the tile kernel: Stan's own termination codes,
    objective within Stan's stall band of the oracle's Stan endpoint, and
    the objective/gradient the tile evaluates equal to the per-series K2 at
    the endpoint (checked through the fitted f)."""
    e, g, ds, Y, Yd = _setup(32)
    fit = e.fit(g, Yd, polish=False, tile_min_series=1)
    st = fit.status.cpu().numpy()
    assert np.all(np.isin(st, [0, 10, 20, 21, 30, 31])), st
    th = fit.theta
    _, ys, _, _, _ = e.prepare(g, Yd)
    f2, _ = e.objective_grad(g, ys, th)
    f, f2 = fit.f.cpu().numpy(), f2.cpu().numpy()
    assert np.all(np.abs(f - f2) <= 1e-11 * np.abs(f2))      # the tile's f at its endpoint
    for s in range(0, 32, 4):
        stp = po.build_problem(ds, Y[s])
        _, fo, *_ = so.fit_setup(stp)
        assert abs(f[s] - fo) <= 2e-4 * abs(fo), (s, f[s], fo)
        fo2, go, _ = so.objective(stp.problem, th[s].cpu().numpy())
        assert abs(fo2 - f[s]) <= 1e-11 * abs(fo2)


def test_tile_flat_growth_and_short_grid():
    """Flat growth (trend = m) and a 730-day grid through the tile kernel vs
    the per-series path: same certified MAP."""
    ds = synthetic.daily_dates("2016-01-01", "2017-12-30")
    e, g, ds, Y, Yd = _setup(20, growth="flat", ds=ds, config_index=3)
    ft = e.fit(g, Yd, tile_min_series=1)
    fs = e.fit(g, Yd, tile_min_series=-1)
    assert np.all(ft.status.cpu().numpy() == fs.status.cpu().numpy())
    f_t, f_s = ft.f.cpu().numpy(), fs.f.cpu().numpy()
    assert np.all(np.abs(f_t - f_s) <= 1e-9 * np.abs(f_s))


def test_tile_default_size_matches_per_series():
    """at the size where K3T runs by default
    (n = 4096 >= tile_min_series = 2048, configs[2]'s generator, the
    persistent schedule with slot refills) the default fit (warm-up hand-off
    to the polish, whose first step is LM-damped) certifies the same MAP as
    Stan's full run + polish (fit_mode stan_map) for the tiled and the
    per-series first pass; their forecasts agree within 1e-6 y_scale;
    refits are bitwise reproducible."""
    n = 4096
    e, g, ds, Y, Yd = _setup(n)
    ft = e.fit(g, Yd)                       # default: tiled first pass
    ft2 = e.fit(g, Yd)
    fs = e.fit(g, Yd, tile_min_series=-1)   # per-series kernel
    fm = e.fit(g, Yd, stan_faithful=True, tile_min_series=-1)
    f_m = fm.f.cpu().numpy()
    for name, fit in (("tile", ft), ("series", fs)):
        st = fit.status.cpu().numpy()
        assert np.all(st == 70), (name, np.unique(st, return_counts=True))
        rel = (fit.f.cpu().numpy() - f_m) / np.abs(f_m)
        assert np.all(rel <= 1e-6), (name, int(np.sum(rel > 1e-6)), float(rel.max()))
        assert np.all(np.abs(rel) <= 1e-9), (name, float(np.abs(rel).max()))
    assert torch.equal(ft.theta, ft2.theta) and torch.equal(ft.f, ft2.f)
    fut = np.concatenate([ds, ds[-1] + synthetic.NS_PER_DAY * np.arange(1, 91)])
    fg = e.predict_grid(ft, fut)
    sid = torch.arange(n, dtype=torch.int32, device="cuda")
    ot = e.predict(ft, fg, seed=0, components=False, series_id=sid)
    os_ = e.predict(fs, fg, seed=0, components=False, series_id=sid)
    ys = ft.y_scale.cpu().numpy()[:, None]
    d = np.abs(ot["yhat"][:, :fg.T].double().cpu().numpy() - os_["yhat"][:, :fg.T].double().cpu().numpy()) / ys
    assert np.all(d <= 1e-6), float(d.max())


@pytest.mark.parametrize("gen", [dict(config_index=1), dict(config_index=2), dict(seed=1001),
                                 dict(seed=1002)])
def test_default_fit_never_worse_than_stan_map(gen):
    """North_star's objective bar, per series, at scale: 4 generator seeds x
    4096 series (1826 days).  The default fit (60-iteration Stan warm-up ->
    polish with an LM-damped first step) is never worse than Stan's full
    L-BFGS run + polish (fit_mode stan_map) by more than 1e-6 relative — 0
    series.  Before the damped first step 8 of these 16384 series certified
    a neighbouring local optimum 3e-5 .. 5e-4 worse (profiles/
    r04a_basin_floor_undamped.json; tools/diag_basin_commit.py shows the
    undamped Newton step from Stan's iteration-60 point jumping basins while
    the polish from iterations 50 or 70 does not)."""
    e = dfa.Engine(0, ProphetConfig.reference())
    ds = synthetic.daily_dates()
    seasons = e.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    n = 4096
    Y = synthetic.sales_matrix(n, ds, **gen)
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    f_def = e.fit(g, Yd).f.cpu().numpy()
    f_sm = e.fit(g, Yd, stan_faithful=True).f.cpu().numpy()
    rel = (f_def - f_sm) / np.abs(f_sm)
    assert int(np.sum(rel > 1e-6)) == 0, (np.flatnonzero(rel > 1e-6), float(rel.max()))
