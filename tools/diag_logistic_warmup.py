"""Diagnostic: configs[4]-shaped fits (hourly T = 8760, logistic + cap,
daily + weekly + yearly + 10 holidays/yr, P = 72).  Reference = Stan's full
L-BFGS run then the polish (what fit_mode 'map' does for logistic growth
today); candidates = a warm-up of W iterations (and 3W/2 evaluations) handed
to the polish.  Counts series whose certified objective is worse than the
reference by > 1e-9 relative (a different basin) and the fit kernels' time.
Run on the GPU box: python tools/diag_logistic_warmup.py [n]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import holidays as H, synthetic  # noqa: E402
from distributed_forecasting_amd.engine import ProphetConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cfg = ProphetConfig.reference()
cfg.growth = "logistic"
ds = synthetic.hourly_dates(n_hours=8760)
seasons = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
hol = H.holiday_spec(H.synthetic_holidays([2017, 2018]), cfg.holidays_prior_scale, cfg.seasonality_mode)
eng = dfa.Engine(0, cfg)
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=hol)
dev = torch.device("cuda", 0)
sets = []
for k in range(2):
    Y, cap = synthetic.saturating_matrix(n, ds, seed=777 + k)
    Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device=dev)
    Yd[:, :grid.T] = torch.from_numpy(Y).to(dev)
    cd = torch.zeros_like(Yd)
    cd[:, :grid.T] = torch.from_numpy(cap).to(dev)
    sets.append((Yd, cd))


def run(**opt):
    fs, ms, ne, st = [], 0.0, [], []
    for Yd, cd in sets:
        eng.ctx.set_timing(True)
        fit = eng.fit(grid, Yd, cap=cd, **opt)
        ks = eng.ctx.read_timings()
        eng.ctx.set_timing(False)
        ms += sum(m for nm, m, _ in ks if nm.startswith("k_fit") or nm.startswith("k_polish"))
        fs.append(fit.f.clone())
        ne.append(fit.n_eval.cpu().numpy())
        st.append(fit.status.cpu().numpy())
    return fs, ms, np.concatenate(ne), np.concatenate(st)


ref, ms0, ne0, st0 = run()
print(f"reference (Stan full + polish): {ms0:.1f} ms for {2 * n} series, n_eval mean {ne0.mean():.0f} "
      f"max {ne0.max()}, certified {np.mean(st0 == 70):.4f}", flush=True)
for W in (60, 100, 150, 200, 300):
    fs, ms, ne, st = run(lbfgs_warmup=W, lbfgs_warmup_evals=(3 * W) // 2)
    worse = sum(int(((f - r) > 1e-9 * r.abs()).sum().item()) for f, r in zip(fs, ref))
    better = sum(int(((r - f) > 1e-9 * r.abs()).sum().item()) for f, r in zip(fs, ref))
    print(f"warm-up {W} iters / {(3 * W) // 2} evals: {ms:.1f} ms, n_eval mean {ne.mean():.0f} max {ne.max()}, "
          f"certified {np.mean(st == 70):.4f}, worse basin {worse} / {2 * n}, better {better}", flush=True)
