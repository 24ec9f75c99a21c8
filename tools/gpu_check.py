"""Quick end-to-end GPU check against the CPU oracle (dev tool; tests/ has the gated version)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402
from oracle import prophet_oracle as po, stan_oracle as so  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
cfg = eng.config
seasons = cfg.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
torch.cuda.synchronize()
setup = po.build_problem(ds, Y[0])
pb = setup.problem
t_g = grid.t[:grid.T].cpu().numpy()
print("t bitexact:", np.array_equal(t_g, setup.hist.t))
print("cp_idx:", grid.cp_idx.cpu().numpy().tolist() == setup.cp_idx.tolist())
print("t_change bitexact:", np.array_equal(grid.t_change.cpu().numpy(), pb.t_change))
XT = grid.XT.view(grid.K, grid.T_pad)[:, :grid.T].cpu().numpy()
print("X max abs diff:", np.abs(XT.T - pb.X).max())
seg = grid.seg[:grid.T].cpu().numpy()
print("seg ok:", np.array_equal(seg, pb.A.sum(1).astype(int)))

Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
y_scale, y_scaled, theta0, status, _ = eng.prepare(grid, Yd)
torch.cuda.synchronize()
print("y_scale ok:", np.allclose(y_scale.cpu().numpy(), np.abs(Y).max(1)))
print("theta0 diff:", np.abs(theta0[0].cpu().numpy() - setup.theta0).max())

# objective / gradient at a random point
rng = np.random.default_rng(0)
th = np.tile(setup.theta0, (n, 1))
th[:, 2:2 + pb.S] = rng.normal(0, 0.02, (n, pb.S))
th[:, 3 + pb.S:] = rng.normal(0, 0.02, (n, pb.K))
th[:, 2 + pb.S] = -1.5
f_g, g_g = eng.objective_grad(grid, y_scaled, torch.from_numpy(th).cuda())
torch.cuda.synchronize()
worst_f = worst_g = 0.0
for s in range(n):
    sp = po.build_problem(ds, Y[s]).problem
    th_s = th[s].copy()
    th_s[:2] = po.build_problem(ds, Y[s]).theta0[:2] if False else th_s[:2]
    f_o, g_o, _ = so.objective(sp, th_s)
    worst_f = max(worst_f, abs(f_g[s].item() - f_o) / abs(f_o))
    worst_g = max(worst_g, np.abs(g_g[s].cpu().numpy() - g_o).max() / np.abs(g_o).max())
print(f"objective rel err {worst_f:.2e}  grad rel err {worst_g:.2e}")

for polish in (False, True):
    t0 = time.time()
    fit = eng.fit(grid, Yd, polish=polish)
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"fit polish={polish}: {dt*1e3:.1f} ms  status={fit.status.cpu().numpy().tolist()}")
    print("   n_eval", fit.n_eval.cpu().numpy().tolist())
    for s in range(min(n, 6)):
        st = po.build_problem(ds, Y[s])
        if polish:
            th_o, f_o, st_o, it_o, ne_o, fst_o = so.fit_map(st)
        else:
            th_o, f_o, st_o, it_o, ne_o = so.fit_setup(st)
        thg = fit.theta[s].cpu().numpy()
        pt_g = po.predict_point(st, po.params_from_theta(thg, st.problem.S), ds)["yhat"]
        pt_o = po.predict_point(st, po.params_from_theta(th_o, st.problem.S), ds)["yhat"]
        print(f"   s{s}: gpu f={fit.f[s].item():.8f} f_stan={fit.f_stan[s].item():.6f} "
              f"ne={fit.n_eval[s].item()} | oracle f={f_o:.8f} ne={ne_o} st={st_o} | "
              f"rel={(fit.f[s].item()-f_o)/abs(f_o):+.2e} dyhat/ys={np.abs(pt_g-pt_o).max()/st.hist.y_scale:.1e}")

fut = dfa.future_dates(ds, 90)
fg = eng.predict_grid(fit, fut)
t0 = time.time()
out = eng.predict(fit, fg, seed=1)
torch.cuda.synchronize()
print(f"predict {1e3*(time.time()-t0):.1f} ms")
for s in range(min(n, 3)):
    st = po.build_problem(ds, Y[s])
    par = po.params_from_theta(fit.theta[s].cpu().numpy(), st.problem.S)
    pt = po.predict_point(st, par, fut)
    yh = out["yhat"][s, :fg.T].cpu().numpy()
    print(f"   s{s}: yhat rel {np.abs(yh - pt['yhat']).max()/st.hist.y_scale:.2e}", end="")
    mc = po.sample_uncertainty(st, par, fut, n_samples=1000, rng=np.random.default_rng(s))
    lo = out["yhat_lower"][s, :fg.T].cpu().numpy()
    hi = out["yhat_upper"][s, :fg.T].cpu().numpy()
    sd = par.sigma_obs * st.hist.y_scale
    print(f"  lo diff/sd mean {np.mean(lo - mc['yhat_lower'])/sd:+.3f} max {np.abs(lo-mc['yhat_lower']).max()/sd:.3f}"
          f"  hi diff/sd mean {np.mean(hi - mc['yhat_upper'])/sd:+.3f} max {np.abs(hi-mc['yhat_upper']).max()/sd:.3f}")
    tl = out["trend_lower"][s, :fg.T].cpu().numpy()
    th_ = out["trend_upper"][s, :fg.T].cpu().numpy()
    print(f"       future trend lo/hi gpu {tl[-1]:.3f}/{th_[-1]:.3f} oracle {mc['trend_lower'][-1]:.3f}/{mc['trend_upper'][-1]:.3f}")
