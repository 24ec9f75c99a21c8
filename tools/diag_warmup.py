"""Diagnostic: warm-up length vs basin agreement with Stan's full L-BFGS run
(fit_mode 'stan_map' = the reference's optimizer run then the polish) on
2000 Kaggle-shaped series (4 generator seeds x 500), and the configs[1]
fused-kernel time of each setting.  Run on the GPU box."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

ds = synthetic.daily_dates()
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
sets = []
for ci in (1, 5, 6, 7):
    Y = synthetic.sales_matrix(500, ds, config_index=ci)
    Yd = torch.zeros((500, grid.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
    ref = eng.fit(grid, Yd, stan_faithful=True)
    sets.append((Yd, ref.f.clone()))
torch.cuda.synchronize()


def run(**opt):
    worse, ms, nem, nex = 0, [], [], []
    for Yd, fref in sets:
        fit = eng.fit(grid, Yd, **opt)
        torch.cuda.synchronize()
        eng.ctx.set_timing(True)
        for _ in range(3):
            fit = eng.fit(grid, Yd, **opt)
        ks = eng.ctx.read_timings()
        eng.ctx.set_timing(False)
        ms.append(sum(m for n_, m, _ in ks if n_.startswith("k_fit") or n_.startswith("k_polish")) / 3)
        worse += int(((fit.f - fref) > 1e-9 * fref.abs()).sum().item())
        ne = fit.n_eval.cpu().numpy()
        nem.append(ne.mean())
        nex.append(ne.max())
        assert bool((fit.status == 70).all())
    return worse, np.mean(ms), np.mean(nem), np.max(nex)


for W, WE in ((60, 90), (60, 80), (50, 80), (60, 0)):
    w, ms, nem, nex = run(lbfgs_warmup=W, lbfgs_warmup_evals=WE)
    print(f"warmup {W:3d} iters, {WE:3d} evals: worse basin than stan_map {w:2d} / 2000; "
          f"fit {ms:.3f} ms per 500; n_eval mean {nem:.1f} max {nex}", flush=True)
