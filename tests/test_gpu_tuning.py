"""GPU: per-series prior scales (pf_problem.tau_series / sigmas_series) and
the batched hyperparameter search (distributed_forecasting_amd.tuning; the
AutoML ProphetHyperoptEstimator search, notebooks/automl/...:109-123).

  * a batch whose rows carry their own prior scales reaches bit-for-bit the
    fit of per-trial batches run with those scales as the shared config;
  * against the oracle (Stan L-BFGS + exact-MAP polish with the trial's
    changepoint/seasonality prior scales): objective within 1e-9 rel, yhat
    within 1e-6 * y_scale;
  * the search's CV metric table equals per-trial cv_metrics_device runs and
    its best trial is the argmin.
"""
import dataclasses

import numpy as np
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import batch as B, synthetic, tuning
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

pytestmark = pytest.mark.gpu

TRIALS = [dict(changepoint_prior_scale=0.05, seasonality_prior_scale=10.0),
          dict(changepoint_prior_scale=0.5, seasonality_prior_scale=0.01),
          dict(changepoint_prior_scale=0.002, seasonality_prior_scale=3.0)]


def _setup(n, seed):
    ds = synthetic.daily_dates()
    return ds, synthetic.sales_matrix(n, ds, seed=seed)


def _fit(eng, ds, Y, priors=None):
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    Yd = torch.zeros((Y.shape[0], g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(np.ascontiguousarray(Y)).cuda()
    pri = eng.series_priors(g, Y.shape[0], **priors) if priors is not None else None
    return g, eng.fit(g, Yd, priors=pri)


def test_per_series_priors_equal_shared_config_fits():
    ds, Y = _setup(8, 321)
    eng = dfa.Engine(0)
    n, M = Y.shape[0], len(TRIALS)
    Yr = np.tile(Y, (M, 1))
    pri = {k: np.repeat([t[k] for t in TRIALS], n) for k in TRIALS[0]}
    _, fb = _fit(eng, ds, Yr, pri)
    for j, tr in enumerate(TRIALS):
        ej = dfa.Engine(0, dataclasses.replace(eng.config, **tr))
        _, fj = _fit(ej, ds, Y)
        rows = slice(j * n, (j + 1) * n)
        assert torch.equal(fb.theta[rows], fj.theta), j
        assert torch.equal(fb.f[rows], fj.f), j
        assert torch.equal(fb.status[rows], fj.status), j


def test_per_series_priors_vs_oracle():
    ds, Y = _setup(2, 77)
    eng = dfa.Engine(0)
    n, M = Y.shape[0], len(TRIALS)
    Yr = np.tile(Y, (M, 1))
    pri = {k: np.repeat([t[k] for t in TRIALS], n) for k in TRIALS[0]}
    g, fit = _fit(eng, ds, Yr, pri)
    fut = B.future_dates(ds, 90)
    fg = eng.predict_grid(fit, fut)
    yh = eng.predict(fit, fg, n_samples=0, components=False)["yhat"][:, :fg.T].cpu().numpy()
    f = fit.f.cpu().numpy()
    for r in range(M * n):
        tr, s = TRIALS[r // n], r % n
        cfg = dict(po.DEFAULT_CONFIG, **tr)
        st = po.build_problem(ds, Y[s], cfg=cfg)
        th, f_o = so.fit_map(st)[:2]
        assert abs(f[r] - f_o) <= 1e-9 * abs(f_o), (r, f[r], f_o)
        pt = po.predict_point(st, po.params_from_theta(th, st.problem.S), fut)
        assert np.max(np.abs(yh[r] - pt["yhat"])) / st.hist.y_scale <= 1e-6, r


def test_series_priors_validation():
    ds, _ = _setup(1, 1)
    eng = dfa.Engine(0)
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    tau, sig = eng.series_priors(g, 3, changepoint_prior_scale=[0.1, 0.2, 0.3])
    assert tau.cpu().tolist() == [0.1, 0.2, 0.3]
    assert sig.shape == (3, g.K) and bool((sig == 10.0).all())
    with pytest.raises(ValueError):
        eng.series_priors(g, 2, seasonality_prior_scale=[1.0, -1.0])


def test_hyperparameter_search_matches_per_trial_cv():
    ds, Y = _setup(3, 11)
    trials = TRIALS[:2] + [dict(changepoint_prior_scale=0.1, seasonality_prior_scale=1.0,
                                seasonality_mode="additive")]
    res = tuning.hyperparameter_search(0, ds, Y, trials, metric="smape")
    assert res.metrics.shape == (3, 3, len(dfa.CV_METRICS))
    base = dfa.ProphetConfig.reference()
    seasons = base.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    for j, tr in enumerate(trials):
        ej = dfa.Engine(0, dataclasses.replace(base, **tr))
        m = dfa.cv_metrics_device(ej, ds, Y, seasons=seasons).cpu().numpy()
        ok = ~np.isnan(m)
        assert np.array_equal(np.isnan(res.metrics[:, j]), ~ok)
        assert np.allclose(res.metrics[:, j][ok], m[ok], rtol=1e-9, atol=0), j
    col = dfa.CV_METRICS.index("smape")
    assert np.array_equal(res.best_trial, np.argmin(res.metrics[:, :, col], axis=1))
    fits = res.best_fit(0, ds, Y)
    got = np.sort(np.concatenate([idx for idx, _ in fits.values()]))
    assert np.array_equal(got, np.arange(3))
    for mode, (idx, fb) in fits.items():
        assert np.all(fb.fit.status.cpu().numpy() == 70), mode
