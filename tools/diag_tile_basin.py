"""Diagnostic: series whose default (warm-up hand-off) fit certifies a
different local MAP than Stan's full run + polish (fit_mode stan_map), for
the tiled and the per-series first pass and several warm-up caps, on
configs[2]'s generator (n series, 1826 days).
    python tools/diag_tile_basin.py [n] [config_index]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import numpy as np, torch
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
from distributed_forecasting_amd.engine import ProphetConfig
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ci = int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = ProphetConfig.reference()
e = dfa.Engine(0, c)
ds = synthetic.daily_dates()
seasons = c.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Y = synthetic.sales_matrix(n, ds, config_index=ci)
Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :g.T] = torch.from_numpy(Y).cuda()
fm = e.fit(g, Yd, stan_faithful=True, tile_min_series=-1).f.cpu().numpy()   # Stan's full run + polish
fst = e.fit(g, Yd, polish=False, tile_min_series=-1).f.cpu().numpy()        # Stan's endpoint
res = {"n": n, "config_index": ci}
for tm in (None, -1):
    for W, WE in ((60, 90), (60, 120), (80, 120), (100, 150)):
        kw = {"lbfgs_warmup": W, "lbfgs_warmup_evals": WE}
        if tm is not None:
            kw["tile_min_series"] = tm
        torch.cuda.synchronize()
        e.ctx.set_timing(True)
        fit = e.fit(g, Yd, **kw)
        torch.cuda.synchronize()
        ms = sum(v for k, v, _ in e.ctx.read_timings())
        e.ctx.set_timing(False)
        f = fit.f.cpu().numpy()
        rel_m = (f - fm) / np.abs(fm)
        rel_s = (f - fst) / np.abs(fst)
        key = f"{'tile' if tm is None else 'series'} W={W} WE={WE}"
        res[key] = {"worse_than_stan_map_1e-9": int(np.sum(rel_m > 1e-9)),
                    "worse_than_stan_endpoint_1e-6": int(np.sum(rel_s > 1e-6)),
                    "max_rel_vs_stan_endpoint": float(rel_s.max()), "fit_ms": round(ms, 2),
                    "mean_eval": float(fit.n_eval.double().mean())}
        print(key, res[key], flush=True)
print(json.dumps(res))
