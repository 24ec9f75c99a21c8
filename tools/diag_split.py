"""Diagnostic: the configs[1] fit with the fused kernel split into its passes
(PF_SPLIT_POLISH=1: k_fit warm-up, k_polish, k_fit_resume, k_polish_resume as
separate launches), so HIP events time the L-BFGS warm-up and the polish
separately."""
import os
import sys

os.environ["PF_SPLIT_POLISH"] = "1"
import torch  # noqa: E402

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
eng.fit(g, Yd)
torch.cuda.synchronize()
eng.ctx.set_timing(True)
for _ in range(5):
    fit = eng.fit(g, Yd)
ks = eng.ctx.read_timings()
eng.ctx.set_timing(False)
agg = {}
for name, ms, grid in ks:
    a = agg.setdefault(name, [0.0, 0])
    a[0] += ms / 5
    a[1] = grid
print({k: (round(v[0], 4), v[1]) for k, v in agg.items()})
print("certified", float((fit.status == 70).float().mean().item()))
