"""Diagnostic: per-series cost of the warm-up and of the exact-MAP polish at
configs[1] (PF_SPLIT_POLISH=1; every series fitted alone, HIP events), to
see whether the 500-series polish launch is set by a few outliers."""
import os
import sys

os.environ["PF_SPLIT_POLISH"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

ds = synthetic.daily_dates()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :g.T] = torch.from_numpy(Y).cuda()
eng.fit(g, Yd[:1].contiguous())
torch.cuda.synchronize()
fit_ms, pol_ms, ne = np.zeros(n), np.zeros(n), np.zeros(n, np.int64)
eng.ctx.set_timing(True)
for i in range(n):
    f = eng.fit(g, Yd[i:i + 1].contiguous())
    ks = eng.ctx.read_timings()
    fit_ms[i] = sum(m for nm, m, _ in ks if nm == "k_fit")
    pol_ms[i] = sum(m for nm, m, _ in ks if nm.startswith("k_polish"))
    ne[i] = int(f.n_eval[0].item())
eng.ctx.set_timing(False)
for name, v in (("warm-up", fit_ms), ("polish", pol_ms)):
    q = np.quantile(v, [0.5, 0.9, 0.99])
    print(f"{name}: mean {v.mean():.3f} ms, p50 {q[0]:.3f}, p90 {q[1]:.3f}, p99 {q[2]:.3f}, max {v.max():.3f}")
o = np.argsort(pol_ms)[::-1][:8]
print("slowest polish series:", [(int(i), round(float(pol_ms[i]), 3), int(ne[i])) for i in o])
print("corr(polish, n_eval) =", float(np.corrcoef(pol_ms, ne)[0, 1]))
