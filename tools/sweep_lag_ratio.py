"""Diagnostic: the polish's lagged-Hessian rule (pf_fit_opts.polish_lag_ratio)
at the headline shape: 4 generator seeds x n series (1826 days); per ratio,
series worse than stan_map by > 1e-6 / 1e-9 relative, uncertified series, the
fit's kernel time and the 500-series launch time.
    python tools/sweep_lag_ratio.py [n] [out.json]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
from distributed_forecasting_amd.engine import ProphetConfig

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out_path = sys.argv[2] if len(sys.argv) > 2 else None
SEEDS = [dict(config_index=1), dict(config_index=2), dict(seed=1001), dict(seed=1002)]
RATIOS = [1e-2, 3e-2, 1e-1, 3e-1]
e = dfa.Engine(0, ProphetConfig.reference())
ds = synthetic.daily_dates()
seasons = e.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))


def timed_fit(Yd, **kw):
    torch.cuda.synchronize()
    e.ctx.set_timing(True)
    fit = e.fit(g, Yd, **kw)
    torch.cuda.synchronize()
    ms = sum(v for k, v, _ in e.ctx.read_timings() if k.startswith("k_fit") or k.startswith("k_polish"))
    e.ctx.set_timing(False)
    return fit, ms


res = {"n": n, "ratios": {}}
for r in RATIOS:
    res["ratios"][str(r)] = {"worse_1e-6": 0, "worse_1e-9": 0, "uncertified": 0, "ms": [], "ms_500": []}
for gen in SEEDS:
    Y = synthetic.sales_matrix(n, ds, **gen)
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    fm = e.fit(g, Yd, stan_faithful=True).f.cpu().numpy()
    for r in RATIOS:
        d = res["ratios"][str(r)]
        fit, ms = timed_fit(Yd, polish_lag_ratio=r)
        rel = (fit.f.cpu().numpy() - fm) / np.abs(fm)
        d["worse_1e-6"] += int(np.sum(rel > 1e-6))
        d["worse_1e-9"] += int(np.sum(rel > 1e-9))
        d["uncertified"] += int((fit.status != 70).sum().item())
        d["ms"].append(round(ms, 3))
        ms5 = []
        for _ in range(3):
            ms5.append(timed_fit(Yd[:500].contiguous(), polish_lag_ratio=r)[1])
        d["ms_500"].append(round(float(np.median(ms5)), 3))
        print(gen, r, d["worse_1e-6"], d["uncertified"], round(ms, 2), d["ms_500"][-1], flush=True)
print(json.dumps(res))
if out_path:
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
