"""GPU parity with holiday columns (SURVEY.md §8a rows a2/a5/a6 for configs[4]):
holiday indicator columns after the Fourier blocks (UPSTREAM
make_holiday_features, holidays_prior_scale), and P = 3 + S + K > 64 — the
yearly + weekly + daily + 10 holidays layout (K = 44, P = 72) runs the wide
kernel variant with two parameter words per lane.  Against the CPU oracle
(oracle/prophet_oracle.py holiday_features / make_features, stan_lbfgs.c)."""
import numpy as np
import pandas as pd
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import holidays as H, synthetic
from distributed_forecasting_amd.engine import ProphetConfig
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

pytestmark = pytest.mark.gpu

DAILY = [("yearly", 365.25, 10), ("weekly", 7.0, 3)]
HOURLY = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]


def _case(hourly, growth, n=4):
    if hourly:
        ds = synthetic.hourly_dates(n_hours=24 * 120)
        seasons = HOURLY
    else:
        ds = synthetic.daily_dates("2015-01-01", "2016-12-31")
        seasons = DAILY
    years = sorted(set(pd.to_datetime(ds).year)) + [int(pd.to_datetime(ds[-1]).year) + 1]
    hd = H.synthetic_holidays(years)
    spec = H.holiday_spec(hd, 10.0)
    c = ProphetConfig.reference()
    c.growth = growth
    eng = dfa.Engine(0, c)
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=spec)
    if growth == "logistic":
        Y, cap = synthetic.saturating_matrix(n, ds)
    else:
        Y, cap = synthetic.sales_matrix(n, ds, config_index=4), None
    cfg = dict(po.DEFAULT_CONFIG, growth=growth)
    cfg["daily"] = (1.0, 4) if hourly else None
    hfn = lambda d: po.holiday_features(d, hd)[0]  # noqa: E731
    return ds, seasons, hd, spec, eng, g, Y, cap, cfg, hfn


def _dev(grid, A):
    Yd = torch.zeros((A.shape[0], grid.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :grid.T] = torch.from_numpy(A).cuda()
    return Yd


@pytest.mark.parametrize("hourly,growth", [(False, "linear"), (True, "linear"), (True, "logistic")])
def test_objective_gradient(hourly, growth):
    ds, seasons, hd, spec, eng, g, Y, cap, cfg, hfn = _case(hourly, growth)
    K, S = g.K, g.S
    assert K == sum(2 * o for _, _, o in seasons) + 10
    capd = _dev(g, cap) if cap is not None else None
    _, ys, th0, _, cs = eng.prepare(g, _dev(g, Y), capd)
    X = g.XT.view(K, g.T_pad)[:, :g.T].cpu().numpy().T
    Xo = po.make_features(ds, cfg, hfn(ds))[0]
    assert np.max(np.abs(X - Xo)) < 1e-13                      # a2 incl. holiday columns
    rng = np.random.default_rng(7)
    th = th0.cpu().numpy().copy()
    th[:, 2:2 + S] = rng.normal(0, 0.02, (4, S))
    th[:, 3 + S:] = rng.normal(0, 0.05, (4, K))
    th[:, 2 + S] = -1.5
    f, gr = eng.objective_grad(g, ys, torch.from_numpy(th).cuda(), cs)
    f, gr = f.cpu().numpy(), gr.cpu().numpy()
    for s in range(4):
        pb = po.build_problem(ds, Y[s], cfg, cap=None if cap is None else cap[s], holiday_cols_fn=hfn).problem
        assert pb.P == g.K + g.S + 3
        fo, go, _ = so.objective(pb, th[s])
        assert abs(f[s] - fo) <= 1e-12 * abs(fo)
        assert np.max(np.abs(gr[s] - go)) <= 1e-10 * np.max(np.abs(go))


@pytest.mark.parametrize("hourly,growth", [(False, "linear"), (True, "logistic")])
def test_fit_and_forecast(hourly, growth):
    """Exact-MAP polish on the holiday layouts (P = 64 daily linear: warm-up
    hand-off; P = 72 hourly logistic: Stan's full L-BFGS first): every series
    certified, objective <= the oracle's Stan endpoint + 1e-6 and equal to its
    certified MAP within 1e-9; the forecast equals the oracle's predict at the
    GPU's theta, holiday columns included."""
    ds, seasons, hd, spec, eng, g, Y, cap, cfg, hfn = _case(hourly, growth)
    capd = _dev(g, cap) if cap is not None else None
    fit = eng.fit(g, _dev(g, Y), cap=capd)
    f = fit.f.cpu().numpy()
    assert np.all(fit.status.cpu().numpy() == 70)         # certified MAP (P = 64 / 72 polish)
    step = ds[1] - ds[0]
    fut = np.concatenate([ds, ds[-1] + step * np.arange(1, 91)])
    fg = eng.predict_grid(fit, fut)
    capf = None if cap is None else np.repeat(cap[:, :1], len(fut), axis=1)
    out = eng.predict(fit, fg, seed=5, cap=None if capf is None else _dev(fg, capf))
    th = fit.theta.cpu().numpy()
    for s in range(Y.shape[0]):
        setup = po.build_problem(ds, Y[s], cfg, cap=None if cap is None else cap[s], holiday_cols_fn=hfn)
        _, f_m, _, _, _, fo = so.fit_map(setup)
        assert f[s] <= fo + 1e-6 * abs(fo)
        assert abs(f[s] - f_m) <= 1e-9 * abs(f_m), (s, f[s], f_m)
        par = po.params_from_theta(th[s], setup.problem.S)
        pt = po.predict_point(setup, par, fut, cfg, cap=None if capf is None else capf[s], holiday_cols_fn=hfn)
        ysc = setup.hist.y_scale
        yh = out["yhat"][s, :fg.T].double().cpu().numpy()
        assert np.max(np.abs(yh - pt["yhat"])) <= 1e-5 * ysc
        hol = out["holidays"][s, :fg.T].double().cpu().numpy()
        Xh = po.holiday_features(fut, hd)[0]
        assert np.max(np.abs(hol - Xh @ par.beta[-10:])) <= 1e-5
        assert np.all(out["yhat_lower"][s, :fg.T].cpu().numpy() <= yh + 1e-3 * ysc)



def test_prophet_class_holidays():
    """Prophet(holidays=...) host surface: component columns per holiday and
    'holidays' in UPSTREAM's crosstab (sorted) order; forecast vs the oracle
    at the fitted theta."""
    ds = synthetic.daily_dates("2015-01-01", "2016-12-31")
    hd = H.synthetic_holidays([2015, 2016, 2017], n_per_year=4)
    y = synthetic.sales_matrix(1, ds, config_index=4)[0]
    df = pd.DataFrame({"ds": ds.astype("datetime64[ns]"), "y": y})
    m = dfa.Prophet(holidays=hd, seasonality_mode="multiplicative", yearly_seasonality=True,
                    weekly_seasonality=True, daily_seasonality=False)
    m.fit(df)
    fut = m.make_future_dataframe(periods=90)
    fc = m.predict(fut)
    comp = [c for c in fc.columns if c not in ("ds", "trend", "yhat", "yhat_lower", "yhat_upper",
                                               "trend_lower", "trend_upper")
            and not c.endswith(("_lower", "_upper"))]
    assert comp == ["hol00", "hol01", "hol02", "hol03", "holidays", "multiplicative_terms", "weekly",
                    "yearly", "additive_terms"]
    hsum = sum(fc[h] for h in ("hol00", "hol01", "hol02", "hol03"))
    assert np.allclose(fc["holidays"], hsum, atol=1e-6)
    assert np.allclose(fc["multiplicative_terms"], fc["holidays"] + fc["weekly"] + fc["yearly"], atol=1e-5)
    cfg = dict(po.DEFAULT_CONFIG)
    hfn = lambda d: po.holiday_features(d, hd)[0]  # noqa: E731
    setup = po.build_problem(ds, y, cfg, holiday_cols_fn=hfn)
    th = m._batch.fit.theta[0].cpu().numpy()
    pt = po.predict_point(setup, po.params_from_theta(th, setup.problem.S), dfa.future_dates(ds, 90), cfg,
                          holiday_cols_fn=hfn)
    assert np.max(np.abs(fc["yhat"].to_numpy() - pt["yhat"])) <= 1e-5 * setup.hist.y_scale


def test_prophet_json_export_holidays(tmp_path):
    """serialize.model_to_json on a holiday model: one component column per
    holiday plus 'holidays'; json_to_record rebuilds the holiday columns from
    the model's holidays frame, and the imported fit serves the same yhat."""
    import io
    import json
    from distributed_forecasting_amd import serialize
    ds = synthetic.daily_dates("2015-01-01", "2016-12-31")
    hd = H.synthetic_holidays([2015, 2016, 2017], n_per_year=4)
    y = synthetic.sales_matrix(1, ds, config_index=4)[0]
    m = dfa.Prophet(holidays=hd, seasonality_mode="multiplicative", yearly_seasonality=True,
                    weekly_seasonality=True, daily_seasonality=False)
    m.fit(pd.DataFrame({"ds": ds.astype("datetime64[ns]"), "y": y}))
    d = json.loads(serialize.model_to_json(m))
    names = pd.read_json(io.StringIO(d["train_holiday_names"]), typ="series", orient="split")
    assert list(names) == ["hol00", "hol01", "hol02", "hol03"]
    tcc = pd.read_json(io.StringIO(d["train_component_cols"]), orient="table")
    nb = np.shape(d["params"]["beta"])[1]
    assert tcc.shape[0] == nb
    assert tcc["holidays"].sum() == sum(tcc[h].sum() for h in names) == nb - 26
    assert tcc["multiplicative_terms"].sum() == nb
    rec = serialize.json_to_record(json.dumps(d), keys=[3, 4])
    assert list(rec["hol_names"]) == list(m._batch.fit.grid.holidays.names)
    cfg = m.config()
    store = dfa.ParamsStore(str(tmp_path / "hol"), config=cfg)
    store.put_record(rec)
    fut = m.make_future_dataframe(periods=90)
    fc = m.predict(fut)
    out = dfa.ForecastStoreItemModel(store).predict(None, fut.assign(store=3, item=4))
    assert np.allclose(out["yhat"].to_numpy(np.float64), fc["yhat"].to_numpy(), rtol=1e-6, atol=1e-4)


def test_params_store_holiday_fit_roundtrip(tmp_path):
    """A holiday fit persisted with put_batch keeps its holiday columns: the
    served forecast equals the batch's own forecast (theta is read with the
    stride of the full grid, 3 + S + K with the holiday columns); a record
    whose theta width does not match its grid is refused."""
    ds, seasons, hd, spec, eng, g, Y, cap, cfg, hfn = _case(False, "linear", n=3)
    fb = dfa.FittedBatch.fit_dense(eng, ds, Y, seasons=seasons, holidays=spec,
                                   series_ids=np.arange(3, dtype=np.int32))
    keys = np.array([[1, 1], [1, 2], [2, 1]])
    store = dfa.ParamsStore(str(tmp_path / "p"), config=eng.config)
    store.put_batch(fb, keys)
    fut = dfa.future_dates(ds, 90)
    Tf, ref = fb.predict(fut, seed=0, components=False)
    inp = pd.DataFrame({"ds": np.tile(fut.astype("datetime64[ns]"), 3),
                        "store": np.repeat(keys[:, 0], Tf), "item": np.repeat(keys[:, 1], Tf)})
    out = dfa.ForecastStoreItemModel(store, seed=0).predict(None, inp)
    for i, (s, it) in enumerate(keys):
        o = out[(out.store == s) & (out.item == it)]
        for k in ("yhat", "yhat_lower", "yhat_upper"):
            assert np.array_equal(o[k].to_numpy(), ref[k][i, :Tf].cpu().numpy()), k
    rec = dict(fb.to_record(keys))
    for k in [k for k in rec if k.startswith("hol_")]:
        del rec[k]
    with pytest.raises(ValueError, match="3 \\+ S \\+ K"):
        dfa.FittedBatch.from_record(eng, rec)
