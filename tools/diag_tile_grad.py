"""Diagnostic: the first L-BFGS step (-alpha g0) of the tiled kernel vs the
per-series kernel, per parameter (which gradient components differ)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests/golden")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import holidays as H, synthetic  # noqa: E402
from distributed_forecasting_amd.engine import ProphetConfig  # noqa: E402
from make_golden import configs4_inputs  # noqa: E402

np.set_printoptions(linewidth=220, precision=6, suppress=True)


def run(name, c, ds, seasons, Y, cap, hol=None):
    eng = dfa.Engine(0, c)
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=hol)

    def dev(A):
        t = torch.zeros((A.shape[0], g.T_pad), dtype=torch.float64, device="cuda")
        t[:, :g.T] = torch.from_numpy(A).cuda()
        return t
    Yd = dev(Y)
    cd = dev(cap) if cap is not None else None
    _, ys, th0, _, cs = eng.prepare(g, Yd, cd)
    _, g0 = eng.objective_grad(g, ys, th0, cs)
    a = eng.fit(g, Yd, cap=cd, polish=False, tile_min_series=1, max_iter=1)
    b = eng.fit(g, Yd, cap=cd, polish=False, tile_min_series=-1, max_iter=1)
    S = g.S
    np.savez(f"gpurun_out/r03f_{name}.npz", th0=th0.cpu().numpy(), ta=a.theta.cpu().numpy(),
             tb=b.theta.cpu().numpy(), g0=g0.cpu().numpy(), ys=ys[:, :g.T].cpu().numpy(),
             cs=cs[:, :g.T].cpu().numpy() if cs is not None else np.zeros(1),
             t=g.t[:g.T].cpu().numpy(), tc=g.t_change.cpu().numpy(), seg=g.seg[:g.T].cpu().numpy(),
             X=g.XT.view(g.K, g.T_pad)[:, :g.T].cpu().numpy())
    for s in range(min(2, Y.shape[0])):
        da = (a.theta[s] - th0[s]).cpu().numpy()
        db = (b.theta[s] - th0[s]).cpu().numpy()
        gg = -g0[s].cpu().numpy()
        na, nb, ng = da / np.abs(da).max(), db / np.abs(db).max(), gg / np.abs(gg).max()
        bad = np.flatnonzero(np.abs(na - nb) > 1e-6)
        print(f"{name} series {s}: P={len(da)} S={S} K={g.K}; params where tile step != K3 step:", bad)
        print("  tile", na[bad][:40])
        print("  K3  ", nb[bad][:40])
        print("  -g0 ", ng[bad][:40])


c = ProphetConfig.reference()
c.growth = "logistic"
ds = synthetic.daily_dates("2015-01-01", "2016-12-31")
Y, cap = synthetic.saturating_matrix(4, ds)
run("daily-logistic", c, ds, [("yearly", 365.25, 10), ("weekly", 7.0, 3)], Y, cap)
c2 = ProphetConfig.reference()
c2.growth = "logistic"
c2.daily_seasonality = True
dh = synthetic.hourly_dates(n_hours=24 * 60)
Y, cap = synthetic.saturating_matrix(4, dh)
HOURLY = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
run("hourly-logistic", c2, dh, HOURLY, Y, cap)
c3 = ProphetConfig.reference()
c3.daily_seasonality = True
run("hourly-linear", c3, dh, HOURLY, Y, None)
ds4, Y4, cap4, hd, cfg = configs4_inputs()
run("configs4", c2, ds4, HOURLY, Y4[:2], cap4[:2], H.holiday_spec(hd, 10.0))
