"""Dev tool: the post-fit tail of the headline step (500 x 1826 days, exact
intervals): K5 (k_predict_mc) time against its blocks per series
(PF_MC_GX = 1, 2, 4, 8; outputs must be bitwise equal), K4, and the in-sample
metrics kernel, each alone (mean of 20 launches, HIP events).
    python tools/time_tail.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import batch as B, diagnostics, synthetic

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
fit = eng.fit(grid, Yd)
fg = eng.predict_grid(fit, B.future_dates(ds, 90))
sid = torch.arange(n, dtype=torch.int32, device="cuda")


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    acc = {}
    for k, v, _ in eng.ctx.read_timings():
        acc[k] = acc.get(k, 0.0) + v / reps
    eng.ctx.set_timing(False)
    return {k: round(v, 4) for k, v in acc.items()}, out


res = {"n": n}
ref = None
for gx in ("1", "2", "4", "8", ""):
    if gx:
        os.environ["PF_MC_GX"] = gx
    else:
        os.environ.pop("PF_MC_GX", None)
    t, out = timed(lambda: eng.predict(fit, fg, seed=1, series_id=sid, components=False))
    o = {k: v.clone() for k, v in out.items()}
    if ref is None:
        ref = o
    same = all(torch.equal(ref[k][:, :fg.T], o[k][:, :fg.T]) for k in ref)
    res[f"gx={gx or 'default'}"] = {**t, "bitwise_equal_gx1": same}
    print(gx, res[f"gx={gx or 'default'}"], flush=True)
t, met = timed(lambda: diagnostics.insample_metrics(eng, Yd[:, :grid.T], ref["yhat"], ref["yhat_lower"],
                                                    ref["yhat_upper"], mdape=False))
res["insample_metrics_fast"] = t
t, met2 = timed(lambda: diagnostics.insample_metrics(eng, Yd[:, :grid.T], ref["yhat"], ref["yhat_lower"],
                                                     ref["yhat_upper"], mdape=True))
res["insample_metrics_all"] = t
print(json.dumps(res))
