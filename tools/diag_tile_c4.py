"""Diagnostic: configs[4] golden series (T = 8760, logistic, P = 72) through
the tiled first pass vs the per-series kernel: Stan-phase endpoints
(objective, status, evaluations), the certified MAP after the polish, and
the gold fixture's Stan endpoint / MAP."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests/golden")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import holidays as H  # noqa: E402
from distributed_forecasting_amd.engine import ProphetConfig  # noqa: E402
from make_golden import configs4_inputs  # noqa: E402

ds, Y, cap, hd, cfg = configs4_inputs()
with np.load("tests/golden/golden_configs4.npz", allow_pickle=False) as z:
    gold = {k: z[k] for k in z.files}
spec = H.holiday_spec(hd, 10.0)
c = ProphetConfig.reference()
c.growth = "logistic"
c.daily_seasonality = True
eng = dfa.Engine(0, c)
seasons = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=spec)


def dev(A):
    t = torch.zeros((A.shape[0], g.T_pad), dtype=torch.float64, device="cuda")
    t[:, :g.T] = torch.from_numpy(A).cuda()
    return t


Yd, cd = dev(Y), dev(cap)
np.set_printoptions(linewidth=200, precision=10)
print("gold f_stan ", gold["f_stan"], "n_eval", gold["n_eval_stan"], "status", gold["status_stan"])
print("gold f_map  ", gold["f_map"])
for tm in (-1, 1):
    for pol in (False, True):
        fit = eng.fit(g, Yd, cap=cd, polish=pol, tile_min_series=tm)
        tag = f"{'tile' if tm == 1 else 'K3  '} polish={pol}"
        print(tag, "f", fit.f.cpu().numpy(), "\n   f_stan", fit.f_stan.cpu().numpy(), "\n   st",
              fit.status.cpu().numpy(), "n_eval", fit.n_eval.cpu().numpy())
        if not pol:
            _, ys, _, _, cs = eng.prepare(g, Yd, cd)
            f2, gr = eng.objective_grad(g, ys, fit.theta, cs)
            print("   K2 f at endpoint - fit f:", (f2 - fit.f).cpu().numpy(),
                  "|g|inf", gr.abs().max(1).values.cpu().numpy())

# trajectories: Stan phase capped at k iterations, tile vs per-series
print("trajectory (max_iter = k): max |theta_tile - theta_K3| per series")
for k in (1, 2, 3, 5, 8, 12, 20, 40, 80):
    a = eng.fit(g, Yd, cap=cd, polish=False, tile_min_series=1, max_iter=k)
    b = eng.fit(g, Yd, cap=cd, polish=False, tile_min_series=-1, max_iter=k)
    d = (a.theta - b.theta).abs().max(1).values.cpu().numpy()
    print(k, d, "n_eval", a.n_eval.cpu().numpy(), b.n_eval.cpu().numpy())
