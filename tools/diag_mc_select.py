"""Diagnostic: k_predict_mc time in sample mode with the threshold selection
vs the general selection (PF_MC_GENERAL_SELECT=1), n series x T days."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, batch as B
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
cfg_i = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ds = synthetic.daily_dates() if cfg_i != 3 else synthetic.daily_dates("2016-01-01", "2017-12-30")
Y = synthetic.sales_matrix(n, ds, config_index=cfg_i)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
fit = eng.fit(grid, Yd)
fg = eng.predict_grid(fit, B.future_dates(ds, 90))
for general in ("0", "1", "0", "1"):
    os.environ["PF_MC_GENERAL_SELECT"] = general
    eng.predict(fit, fg, seed=1, interval_method="sample"); torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    eng.predict(fit, fg, seed=1, interval_method="sample"); torch.cuda.synchronize()
    ms = {k: v for k, v, _ in eng.ctx.read_timings()}
    eng.ctx.set_timing(False)
    print(f"general={general} k_predict_mc {ms.get('k_predict_mc', float('nan')):.3f} ms")
