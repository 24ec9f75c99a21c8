"""Diagnostic: k_predict_det / k_predict_mc time split (500 x 1826, 90-day
horizon): intervals on (N = 1000) vs off (N = 0), exact vs sample."""
import sys

import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

ds = synthetic.daily_dates()
n = 500
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :g.T] = torch.from_numpy(Y).cuda()
fit = eng.fit(g, Yd)
fg = eng.predict_grid(fit, dfa.future_dates(ds, 90))
for ns, comp in ((1000, False), (0, False), (1000, True)):
    eng.predict(fit, fg, n_samples=ns, components=comp)
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    for _ in range(10):
        eng.predict(fit, fg, n_samples=ns, components=comp)
    ks = eng.ctx.read_timings()
    eng.ctx.set_timing(False)
    agg = {}
    for name, ms, _ in ks:
        agg[name] = agg.get(name, 0.0) + ms / 10
    print(f"n_samples={ns} components={comp}: " + ", ".join(f"{k} {v:.4f} ms" for k, v in agg.items()))
