"""CPU: the oracle against the known-answer tests of SURVEY.md §8c and the
committed golden fixtures (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from distributed_forecasting_amd import synthetic
from oracle import prophet_oracle as po
from oracle import stan_oracle as so

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NSD = po.NS_PER_DAY

KAT_CP = {
    1826: [58, 117, 175, 233, 292, 350, 409, 467, 525, 584, 642, 700, 759, 817, 875, 934, 992,
           1050, 1109, 1167, 1226, 1284, 1342, 1401, 1459],
    730: [23, 47, 70, 93, 117, 140, 163, 187, 210, 233, 257, 280, 303, 326, 350, 373, 396, 420,
          443, 466, 490, 513, 536, 560, 583],
    8760: [280, 561, 841, 1121, 1401, 1682, 1962, 2242, 2523, 2803, 3083, 3363, 3644, 3924, 4204,
           4484, 4765, 5045, 5325, 5606, 5886, 6166, 6446, 6727, 7007],
    1016: [32, 65, 97, 130, 162, 195, 227, 260, 292, 324, 357, 389, 422, 454, 487, 519, 551, 584,
           616, 649, 681, 714, 746, 779, 811],
    1376: [44, 88, 132, 176, 220, 264, 308, 352, 396, 440, 484, 528, 571, 615, 659, 703, 747, 791,
           835, 879, 923, 967, 1011, 1055, 1099],
    1736: [55, 111, 166, 222, 277, 333, 388, 444, 499, 555, 610, 666, 721, 777, 832, 888, 943, 999,
           1054, 1110, 1165, 1221, 1276, 1332, 1387],
}


@pytest.mark.parametrize("T", sorted(KAT_CP))
def test_changepoint_kat(T):
    assert po.changepoint_indices(T).tolist() == KAT_CP[T]


def test_changepoint_clamp():
    # hist_size = floor(T*0.8); n_cp+1 > hist_size -> hist_size - 1 changepoints
    assert len(po.changepoint_indices(10)) == 7
    assert len(po.changepoint_indices(2)) == 0


def test_t_bit_exact_regular_grid():
    ds = synthetic.daily_dates()
    h = po.setup_history(ds, np.arange(len(ds), dtype=float))
    T = len(ds)
    assert np.array_equal(h.t, np.arange(T) / (T - 1))


def test_days_since_epoch():
    ds = synthetic.daily_dates()
    d = po.days_since_epoch(ds)
    assert d[0] == 15706 and d[-1] == 17531
    assert np.array_equal(d, np.arange(15706, 17532))


def test_cv_cutoffs():
    ds = synthetic.daily_dates()
    cut = po.generate_cutoffs(ds, 90 * NSD, 730 * NSD, 360 * NSD)
    assert [(c - ds[0]) // NSD for c in cut] == [1015, 1375, 1735]


def test_percentile_positions():
    lo, hi = po.percentile_positions(1000, 0.95)
    assert abs(lo - 24.975) < 1e-9 and abs(hi - 974.025) < 1e-9


def _random_theta(pb, rng):
    th = np.zeros(pb.P)
    th[0], th[1] = 0.3, 0.4
    th[2:2 + pb.S] = rng.normal(0, 0.02, pb.S)
    th[2 + pb.S] = -1.5
    th[3 + pb.S:] = rng.normal(0, 0.05, pb.K)
    return th


def test_gradient_vs_finite_differences():
    ds = synthetic.daily_dates()
    y = synthetic.sales_matrix(1, ds)[0]
    pb = po.build_problem(ds, y).problem
    rng = np.random.default_rng(1)
    th = _random_theta(pb, rng)
    th[2:2 + pb.S] += np.sign(th[2:2 + pb.S]) * 0.01   # keep |delta| away from the kink
    f, g = po.objective(pb, th)[:2]
    h = 1e-6
    fd = np.empty(pb.P)
    for i in range(pb.P):
        e = np.zeros(pb.P); e[i] = h
        fd[i] = (po.objective(pb, th + e)[0] - po.objective(pb, th - e)[0]) / (2 * h)
    assert np.max(np.abs(fd - g)) / np.max(np.abs(g)) < 1e-7


def test_c_objective_matches_numpy():
    ds = synthetic.daily_dates()
    y = synthetic.sales_matrix(1, ds)[0]
    pb = po.build_problem(ds, y).problem
    th = _random_theta(pb, np.random.default_rng(2))
    f1, g1 = po.objective(pb, th)[:2]
    f2, g2, _ = so.objective(pb, th)
    assert abs(f1 - f2) <= 1e-12 * abs(f1)
    assert np.max(np.abs(g1 - g2)) <= 1e-10 * np.max(np.abs(g1))


def test_map_certified(golden_ref):
    """KAT 9: the engine-semantics fit (Stan L-BFGS + exact-MAP polish) is at
    least as good as a certified scipy L-BFGS-B optimum, and the Stan phase
    stops within 1e-4 relative of it (its stall at the L1 kink)."""
    ds = golden_ref["ds_ns"]
    for s in range(2):
        st = po.build_problem(ds, golden_ref["Y"][s])
        th_c, f_c = so.certify(st.problem, golden_ref["theta_stan"][s])
        f_map = golden_ref["f_map"][s]
        assert f_map <= f_c + 1e-9 * abs(f_c)
        assert golden_ref["f_stan"][s] <= f_c + 1e-4 * abs(f_c)


def test_golden_reproduces(golden_ref):
    """The oracle still produces the committed fixture (regression pin)."""
    ds = golden_ref["ds_ns"]
    st = po.build_problem(ds, golden_ref["Y"][0])
    assert st.cp_idx.tolist() == golden_ref["cp_idx"].tolist() == KAT_CP[1826]
    assert np.array_equal(st.problem.t_change, golden_ref["t_change"])
    th, f, status, it, ne = so.fit_setup(st)
    assert ne == golden_ref["n_eval_stan"][0] and status == golden_ref["status_stan"][0]
    assert np.array_equal(th, golden_ref["theta_stan"][0])
    th_m = so.fit_map(st)[0]
    assert np.max(np.abs(th_m - golden_ref["theta_map"][0])) < 1e-9
    pt = po.predict_point(st, po.params_from_theta(th_m, st.problem.S), golden_ref["fut_ns"])
    assert np.max(np.abs(pt["yhat"] - golden_ref["yhat"][0])) < 1e-8


def test_constant_series(golden_edge):
    assert int(golden_edge["const_status"]) == 50
    th = golden_edge["const_theta"]
    S = 25
    assert abs(np.exp(th[2 + S]) - 1e-9) < 1e-20
    assert np.all(th[2:2 + S] == 0) and np.all(th[3 + S:] == 0)


def test_noise_free_linear(golden_edge):
    ds = synthetic.daily_dates()
    st = po.build_problem(ds, golden_edge["lin_y"])
    par = po.params_from_theta(golden_edge["lin_theta"], st.problem.S)
    assert np.max(np.abs(par.delta)) < 1e-3
    pt = po.predict_point(st, par, ds)
    assert np.max(np.abs(pt["yhat"] - golden_edge["lin_y"])) / st.hist.y_scale < 1e-3


def test_rolling_mean_by_h_small():
    # UPSTREAM sweep by hand: h groups {1:[1,3], 2:[5], 3:[7,9]}, w = 2
    hs, v = po.rolling_mean_by_h(np.array([1., 3., 5., 7., 9.]), np.array([1, 1, 2, 3, 3]), 2)
    assert hs.tolist() == [1, 2, 3]
    assert np.allclose(v, [2.0, 3.5, 8.0])   # h=2: (5 + 4 - 1 * 4/2) / 2


def test_order_statistic_spacings_match_sampling():
    """Math behind PF_INTERVAL_EXACT (csrc/pf_ostat.h): the joint law of the
    normal order statistics at ranks (25, 26, 975, 976) of N = 1000 draws,
    built from Gamma spacings + the inverse normal CDF, equals brute-force
    sorting, checked through np.percentile(·, 2.5 / 97.5) ('linear')."""
    from scipy import stats
    from scipy.special import ndtri
    N, M = 1000, 6000
    rng = np.random.default_rng(20261016)
    Z = rng.standard_normal((M, N))
    bl, bh = np.percentile(Z, 2.5, axis=1), np.percentile(Z, 97.5, axis=1)
    ilo, ihi = N * 0.025 + 0.975 - 1, N * 0.975 + 0.025 - 1
    klo, khi = int(ilo), int(ihi)
    r = [klo + 1, klo + 2, khi + 1, khi + 2]
    shapes = [r[0], r[1] - r[0], r[2] - r[1], r[3] - r[2], N + 1 - r[3]]
    G = np.stack([rng.gamma(s, size=M) for s in shapes], 1)
    U = np.cumsum(G, 1)[:, :4] / G.sum(1)[:, None]
    z = ndtri(U)
    el = z[:, 0] + (z[:, 1] - z[:, 0]) * (ilo - klo)
    eh = z[:, 2] + (z[:, 3] - z[:, 2]) * (ihi - khi)
    assert stats.ks_2samp(bl, el).pvalue > 1e-3
    assert stats.ks_2samp(bh, eh).pvalue > 1e-3
    assert stats.ks_2samp(bh - bl, eh - el).pvalue > 1e-3


def test_rolling_median_by_h_small():
    """Known answers worked by hand from UPSTREAM rolling_median_by_h."""
    x, h = np.array([1., 3., 5., 7., 9.]), np.array([1, 1, 2, 3, 3])
    hs, v = po.rolling_median_by_h(x, h, 2)
    assert hs.tolist() == [1, 2, 3] and v.tolist() == [2.0, 4.0, 8.0]
    hs, v = po.rolling_median_by_h(x, h, 3)
    assert hs.tolist() == [2, 3] and v.tolist() == [3.0, 7.0]


def test_oracle_sanitizers():
    """The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer
    (host only): objective, Stan L-BFGS, Hessians and the damped polish for
    linear, logistic and flat growth (oracle/asan_check.c)."""
    import shutil
    import subprocess
    if shutil.which("make") is None or shutil.which("cc") is None:
        pytest.skip("no host toolchain")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert r.stdout.count("cert 1") == 3, r.stdout
