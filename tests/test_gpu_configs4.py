"""GPU parity at BASELINE.json configs[4]'s own shape (SURVEY.md §8a rows
a3/a5/a6/a7): hourly series x 8760 steps, logistic growth with cap, yearly +
weekly + daily seasonality + 10 holidays/year, P = 3 + 25 + 44 = 72 (the wide
two-words-per-lane kernels, one workgroup per CU in LDS).

Checked against the CPU oracle and its committed fixture
(tests/golden/golden_configs4.npz, tests/golden/make_golden.py configs4):
  * changepoint indices bit-exact with the T = 8760 known answer;
  * objective and gradient within 1e-12 / 1e-10 of orc_objective;
  * the exact Hessian (pf_hessian, the polish's model: sigmoid and
    logistic_gamma curvature) within 1e-9 of orc_hessian;
  * the fit: every series certified (PF_ST_MAP), objective <= the oracle's
    Stan endpoint + 1e-6 relative, and equal to the oracle's certified MAP
    within 1e-9; yhat within 1e-6 * y_scale of the oracle's forecast at its
    MAP.
"""
import os

import numpy as np
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import holidays as H
from distributed_forecasting_amd.engine import ProphetConfig
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

pytestmark = pytest.mark.gpu

HOURLY = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
KAT_8760 = [280, 561, 841, 1121, 1401, 1682, 1962, 2242, 2523, 2803, 3083, 3363, 3644, 3924,
            4204, 4484, 4765, 5045, 5325, 5606, 5886, 6166, 6446, 6727, 7007]
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_configs4.npz")


def _inputs():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import configs4_inputs
    return configs4_inputs()


@pytest.fixture(scope="module")
def c4():
    ds, Y, cap, hd, cfg = _inputs()
    with np.load(GOLDEN, allow_pickle=False) as z:
        gold = {k: z[k] for k in z.files}
    spec = H.holiday_spec(hd, 10.0)
    c = ProphetConfig.reference()
    c.growth = "logistic"
    c.daily_seasonality = True
    eng = dfa.Engine(0, c)
    g = dfa.build_grid(ds, HOURLY, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=spec)
    hfn = lambda d: po.holiday_features(d, hd)[0]  # noqa: E731
    return dict(ds=ds, Y=Y, cap=cap, hd=hd, cfg=cfg, gold=gold, eng=eng, g=g, hfn=hfn)


def _dev(grid, A):
    Yd = torch.zeros((A.shape[0], grid.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :grid.T] = torch.from_numpy(A).cuda()
    return Yd


def _problem(c, s):
    return po.build_problem(c["ds"], c["Y"][s], c["cfg"], cap=c["cap"][s], holiday_cols_fn=c["hfn"])


def test_grid_changepoints_kat(c4):
    g = c4["g"]
    assert g.T == 8760 and g.K == 44 and g.S == 25
    assert g.cp_idx.cpu().numpy().tolist() == KAT_8760
    assert c4["gold"]["cp_idx"].tolist() == KAT_8760


def test_objective_gradient_hessian(c4):
    eng, g, gold = c4["eng"], c4["g"], c4["gold"]
    _, ys, th0, _, cs = eng.prepare(g, _dev(g, c4["Y"]), _dev(g, c4["cap"]))
    assert np.allclose(th0.cpu().numpy(), gold["theta0"], rtol=1e-13, atol=1e-15)   # a4
    g0max = [np.max(np.abs(so.objective(_problem(c4, s).problem, gold["theta0"][s])[1]))
             for s in range(gold["theta0"].shape[0])]
    for name in ("theta_stan", "theta_map"):
        th = torch.from_numpy(gold[name]).cuda()
        f, gr = eng.objective_grad(g, ys, th, cs)
        Hg = eng.hessian(g, ys, th, cs).cpu().numpy()
        f, gr = f.cpu().numpy(), gr.cpu().numpy()
        for s in range(gold[name].shape[0]):
            pb = _problem(c4, s).problem
            fo, go, _ = so.objective(pb, gold[name][s])
            assert abs(f[s] - fo) <= 1e-12 * abs(fo)
            # near the optimum each gradient entry is the cancellation of
            # 8760 row terms ~1e3x larger: compare on the init's scale
            assert np.max(np.abs(gr[s] - go)) <= 1e-11 * g0max[s], (name, s)
            Ho = so.hessian(pb, gold[name][s])
            assert np.max(np.abs(Hg[s] - Ho)) <= 1e-9 * np.max(np.abs(Ho)), (name, s)


def test_fit_certified_map(c4):
    eng, g, gold = c4["eng"], c4["g"], c4["gold"]
    fit = eng.fit(g, _dev(g, c4["Y"]), cap=_dev(g, c4["cap"]))
    st = fit.status.cpu().numpy()
    f = fit.f.cpu().numpy()
    assert np.all(st == 70), st                                        # PF_ST_MAP
    assert np.all(f <= gold["f_stan"] + 1e-6 * np.abs(gold["f_stan"])), (f, gold["f_stan"])
    assert np.all(np.abs(f - gold["f_map"]) <= 1e-9 * np.abs(gold["f_map"])), (f - gold["f_map"]) / gold["f_map"]
    fut = np.concatenate([c4["ds"], c4["ds"][-1] + (c4["ds"][1] - c4["ds"][0]) * np.arange(1, 91)])
    fg = eng.predict_grid(fit, fut)
    capf = np.repeat(c4["cap"][:, :1], len(fut), axis=1)
    out = eng.predict(fit, fg, seed=1, cap=_dev(fg, capf))
    for s in range(len(f)):
        setup = _problem(c4, s)
        pt = po.predict_point(setup, po.params_from_theta(gold["theta_map"][s], setup.problem.S), fut,
                              c4["cfg"], cap=capf[s], holiday_cols_fn=c4["hfn"])
        yh = out["yhat"][s, :fg.T].double().cpu().numpy()
        assert np.max(np.abs(yh - pt["yhat"])) <= 1e-6 * setup.hist.y_scale + 1e-6 * np.abs(pt["yhat"]).max()
