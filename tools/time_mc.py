"""Dev tool: sample-mode forecast kernel times for one engine build.

    python tools/time_mc.py <lib.so|default> [n]   # configs[3] shape: n x 730 days, 90-day horizon
Prints one JSON line: per-kernel ms (mean of 3 timed predicts)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_forecasting_amd import _lib
if sys.argv[1] != "default":
    _lib.load(os.path.abspath(sys.argv[1]))
import numpy as np, torch
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, batch as B
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
ds = synthetic.daily_dates("2016-01-01", "2017-12-30")
Y = synthetic.sales_matrix(n, ds, config_index=3)
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
    eng.predict(fit, fg, seed=1, interval_method="sample", series_id=sid, components=comp)
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    for _ in range(3):
        eng.predict(fit, fg, seed=1, interval_method="sample", series_id=sid, components=comp)
    torch.cuda.synchronize()
    acc = {}
    for k, v, _ in eng.ctx.read_timings():
        acc[k] = acc.get(k, 0.0) + v / 3
    eng.ctx.set_timing(False)
    res[f"comp{int(comp)}"] = {k: round(v, 3) for k, v in acc.items()}
print(json.dumps({"lib": sys.argv[1], "n": n, **res}))
