"""Diagnostic: how often does the default fit (map:
Stan L-BFGS warm-up handed to the certified polish) end in a worse local MAP
than Stan's full run + polish (stan_map), and how often does Stan's full run +
polish itself end in a worse basin when its initial point moves by 1e-14
(Stan's own rounding sensitivity: its L1-kink termination is chaotic)?

For 4 generator seeds x n series (1826 days, the reference layout), counts of
series with f_a > f_b + tol * |f_b| for
  map        vs stan_map
  stan_map(init k * (1 + 1e-14))  vs stan_map     (the floor)
  stan_map(init m * (1 + 1e-14))  vs stan_map     (the floor, second draw)
  stan_map(per-series kernel)     vs stan_map (tiled first pass)
and the violating series' details.
    python tools/diag_basin_floor.py [n] [out.json]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
from distributed_forecasting_amd.engine import ProphetConfig

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out_path = sys.argv[2] if len(sys.argv) > 2 else None
SEEDS = [("config_index=1", dict(config_index=1)), ("config_index=2", dict(config_index=2)),
         ("seed=1001", dict(seed=1001)), ("seed=1002", dict(seed=1002))]
e = dfa.Engine(0, ProphetConfig.reference())
ds = synthetic.daily_dates()
seasons = e.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))


def pert(col):
    def f(th):
        th[:, col] *= 1.0 + 1e-14
    return f


def run(Yd, **kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fit = e.fit(g, Yd, **kw)
    torch.cuda.synchronize()
    return fit, (time.perf_counter() - t0) * 1e3


res = {"n": n, "T": len(ds), "seeds": {}}
tot = {}
for name, kw in SEEDS:
    Y = synthetic.sales_matrix(n, ds, **kw)
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    fits = {}
    fits["stan_map"], t_sm = run(Yd, stan_faithful=True)
    fits["stan_map_pk"], _ = run(Yd, stan_faithful=True, init=pert(0))
    fits["stan_map_pm"], _ = run(Yd, stan_faithful=True, init=pert(1))
    fits["stan_map_series"], _ = run(Yd, stan_faithful=True, tile_min_series=-1)
    fits["map"], t_map = run(Yd)
    fits["stan"], _ = run(Yd, polish=False)
    f = {k: v.f.cpu().numpy() for k, v in fits.items()}
    st = {k: v.status.cpu().numpy() for k, v in fits.items()}
    ref = f["stan_map"]
    r = {"ms_stan_map": round(t_sm, 2), "ms_map": round(t_map, 2)}
    for k in ("map", "stan_map_pk", "stan_map_pm", "stan_map_series"):
        rel = (f[k] - ref) / np.abs(ref)
        for tol in (1e-6, 1e-9):
            c = int(np.sum(rel > tol))
            r[f"{k}_worse_{tol:g}"] = c
            tot[f"{k}_worse_{tol:g}"] = tot.get(f"{k}_worse_{tol:g}", 0) + c
        r[f"{k}_better_1e-6"] = int(np.sum(rel < -1e-6))
        r[f"{k}_max_rel"] = float(rel.max())
        r[f"{k}_certified"] = float(np.mean(st[k] == 70))
    # the best of Stan's three runs: is map worse than every one of them?
    best = np.minimum.reduce([f["stan_map"], f["stan_map_pk"], f["stan_map_pm"], f["stan_map_series"]])
    worst = np.maximum.reduce([f["stan_map"], f["stan_map_pk"], f["stan_map_pm"], f["stan_map_series"]])
    r["stan_runs_spread_gt_1e-6"] = int(np.sum((worst - best) / np.abs(best) > 1e-6))
    r["map_worse_than_all_stan_runs_1e-6"] = int(np.sum((f["map"] - worst) / np.abs(worst) > 1e-6))
    viol = np.flatnonzero((f["map"] - ref) / np.abs(ref) > 1e-6)
    r["map_violators"] = [{"s": int(s), "rel": float((f["map"][s] - ref[s]) / abs(ref[s])),
                           "rel_vs_stan_endpoint": float((f["map"][s] - f["stan"][s]) / abs(f["stan"][s])),
                           "n_eval_map": int(fits["map"].n_eval[s]), "n_eval_stan": int(fits["stan_map"].n_eval[s]),
                           "rel_pk": float((f["stan_map_pk"][s] - ref[s]) / abs(ref[s])),
                           "rel_pm": float((f["stan_map_pm"][s] - ref[s]) / abs(ref[s]))}
                          for s in viol]
    res["seeds"][name] = r
    print(name, json.dumps(r), flush=True)
res["total"] = tot
print(json.dumps(res))
if out_path:
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
