"""Diagnostic: how the configs[1] fused fit launch (k_fit_polish, 500
series) is set by its slowest series.  Prints the n_eval distribution, the
status mix, and the kernel time of the full batch vs the batch without its
slowest series (HIP events), and a warm-up sweep of the tail.
Run on the GPU box: python tools/diag_tail.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

ds = synthetic.daily_dates()
n = 500
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))


def run(rows, reps=5, **opt):
    Yd = torch.zeros((len(rows), grid.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :grid.T] = torch.from_numpy(Y[rows]).cuda()
    fit = eng.fit(grid, Yd, **opt)
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    for _ in range(reps):
        fit = eng.fit(grid, Yd, **opt)
    ks = eng.ctx.read_timings()
    eng.ctx.set_timing(False)
    fk = [ms for name, ms, _ in ks if name.startswith("k_fit") or name.startswith("k_polish")]
    return fit, sum(fk) / reps


rows = np.arange(n)
fit, ms = run(rows)
ne = fit.n_eval.cpu().numpy()
st = fit.status.cpu().numpy()
print(f"all 500: fit kernels {ms:.3f} ms; n_eval mean {ne.mean():.1f} p50 {np.median(ne):.0f} "
      f"p90 {np.quantile(ne, .9):.0f} p99 {np.quantile(ne, .99):.0f} max {ne.max()}")
print("status:", dict(zip(*np.unique(st, return_counts=True))))
print("n_eval histogram (bins of 10):", np.histogram(ne, bins=np.arange(0, ne.max() + 11, 10))[0].tolist())
order = np.argsort(ne)
for drop in (5, 25, 50, 100):
    keep = np.sort(order[:n - drop])
    _, ms2 = run(keep)
    print(f"without the {drop} slowest (n_eval <= {ne[order[n - drop - 1]]}): {ms2:.3f} ms")
for w in (30, 40, 50, 60):
    f2, ms3 = run(rows, lbfgs_warmup=w)
    ne2 = f2.n_eval.cpu().numpy()
    d = (f2.f - fit.f).abs() / fit.f.abs()
    print(f"warmup {w}: {ms3:.3f} ms, n_eval mean {ne2.mean():.1f} max {ne2.max()}, "
          f"certified {(f2.status == 70).float().mean().item():.3f}, "
          f"worse than W=60 by >1e-9 rel: {int((d > 1e-9).sum().item())}")
