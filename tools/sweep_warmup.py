"""Dev tool: L-BFGS warm-up length vs fit+polish time and certification."""
import sys, time
import numpy as np, torch
sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ds = synthetic.daily_dates(); Y = synthetic.sales_matrix(n, ds, config_index=1)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
ref = eng.fit(grid, Yd, stan_faithful=True).f.clone()   # full Stan run + polish: Stan's basin
for spec in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["30", "40", "60"]):
    W, E = (int(x) for x in (spec.split(":") + ["0"])[:2])
    ts = []
    for rep in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        fit = eng.fit(grid, Yd, lbfgs_warmup=W, lbfgs_warmup_evals=E)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    st = fit.status.cpu().numpy()
    d = ((fit.f - ref) / ref.abs()).cpu().numpy()   # > 0: worse than Stan's basin
    print(f"W={W:3d} E={E:3d} fit {1e3*min(ts):.3f} ms  n_eval mean {fit.n_eval.float().mean().item():.1f} max {fit.n_eval.max().item()}"
          f"  certified {np.mean(st == 70):.3f}  (f-f_stan)/|f|: max {d.max():.2e} min {d.min():.2e} #worse>1e-9 {(d > 1e-9).sum()}", flush=True)
