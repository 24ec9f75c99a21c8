"""Run fit + predict a few times on n series (for rocprofv3 kernel traces)."""
import sys, time
import numpy as np, torch
sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
polish = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
fut = dfa.future_dates(ds, 90)
y_scale, y_scaled, theta0, status, _ = eng.prepare(grid, Yd)
for r in range(3):
    torch.cuda.synchronize(); t0 = time.time()
    f_, g_ = eng.objective_grad(grid, y_scaled, theta0)
    torch.cuda.synchronize(); print(f"objgrad (one eval of all {n} series): {1e6*(time.time()-t0):.1f} us", flush=True)
for r in range(reps):
    torch.cuda.synchronize(); t0 = time.time()
    fit = eng.fit(grid, Yd, polish=polish)
    torch.cuda.synchronize(); t1 = time.time()
    fg = eng.predict_grid(fit, fut)
    out = eng.predict(fit, fg, seed=r)
    torch.cuda.synchronize(); t2 = time.time()
    ne = fit.n_eval.cpu().numpy()
    print(f"rep {r}: fit {1e3*(t1-t0):.2f} ms predict {1e3*(t2-t1):.2f} ms  n_eval mean {ne.mean():.0f} max {ne.max()}  "
          f"series/s {n/(t2-t0):.0f}", flush=True)
