"""Dev tool: K5 (k_predict_mc) time at the headline shape (500 x 1826 days,
90-day horizon, exact intervals), mean of 20 timed predicts.
    python tools/time_k5.py <lib.so|default>      (PF_MC_GENERAL_SELECT=1: general selection)"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_forecasting_amd import _lib
if sys.argv[1] != "default":
    _lib.load(os.path.abspath(sys.argv[1]))
import numpy as np, torch
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, batch as B
n = 500
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
fit = eng.fit(grid, Yd)
fg = eng.predict_grid(fit, B.future_dates(ds, 90))
sid = torch.arange(n, dtype=torch.int32, device="cuda")
res = {}
for comp in (False, True):
    eng.predict(fit, fg, seed=1, series_id=sid, components=comp)
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    for _ in range(20):
        eng.predict(fit, fg, seed=1, series_id=sid, components=comp)
    torch.cuda.synchronize()
    acc = {}
    for k, v, _ in eng.ctx.read_timings():
        acc[k] = acc.get(k, 0.0) + v / 20
    eng.ctx.set_timing(False)
    res[f"comp{int(comp)}"] = {k: round(v, 4) for k, v in acc.items()}
print(json.dumps({"lib": sys.argv[1], "general": os.environ.get("PF_MC_GENERAL_SELECT", "0"), **res}))
