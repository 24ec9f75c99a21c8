"""Diagnostic: per-series timeline of the fused launch (k_fit_forecast) at
the headline shape — each workgroup's start, fit end and epilogue end
(s_memrealtime, -DPF_STAMPS build) — to see what sets the launch's makespan:
the distribution of fit times, the epilogue time, and the slowest series'
evaluation / Newton counts.
    python tools/block_timeline.py [n] [config_index] [out.json]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath(os.environ.get("PF_TIMELINE_LIB", "diag_exp/libprophet_hip_timeline.so")))
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 1
out_path = sys.argv[3] if len(sys.argv) > 3 else None
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds, config_index=cfg)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :g.T] = torch.from_numpy(Y).cuda()
fg = dfa.build_grid(dfa.future_dates(ds, 90), seasons, start_ns=g.start_ns, t_scale_ns=g.t_scale_ns,
                    t_change=g.t_change)
res = {"n": n, "runs": []}
buf0 = (ctypes.c_ulonglong * (11 * 4096))()
_lib._lib.pf_debug_blocks(buf0)                      # zero the counters
for rep in range(3):
    fit, out, met, fused = eng.fit_forecast(g, Yd, fg, components=False, metrics="fast")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (11 * 4096))()
    assert _lib._lib.pf_debug_blocks(buf) == 0       # (and zeroes the counters)
    raw = np.array(list(buf), dtype=np.float64).reshape(11, 4096)[:, :n]
    b = raw[:4] / 100.0   # us
    nnewton, npe = raw[4], raw[5]
    hess_us, sweep_us = raw[6] / 100.0, raw[7] / 100.0
    qp_us, ls_us, rs_us = raw[8] / 100.0, raw[9] / 100.0, raw[10] / 100.0
    t0 = b[0].min()
    start, fitend, end, lbend = b[0] - t0, b[1] - t0, b[2] - t0, b[3] - t0
    fit_us, epi_us = fitend - start, end - fitend
    lb_us, pol_us = lbend - start, fitend - lbend
    ne = fit.n_eval.cpu().numpy()
    st = fit.status.cpu().numpy()
    slow = np.argsort(-end)[:8]
    r = {"makespan_us": float(end.max()), "start_max_us": float(start.max()),
         "fit_us": {q: float(np.percentile(fit_us, p)) for q, p in
                    (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
         "epilogue_us": {q: float(np.percentile(epi_us, p)) for q, p in
                         (("p50", 50), ("p90", 90), ("max", 100))},
         "lbfgs_us": {q: float(np.percentile(lb_us, p)) for q, p in
                      (("p50", 50), ("p90", 90), ("max", 100))},
         "polish_us": {q: float(np.percentile(pol_us, p)) for q, p in
                       (("p50", 50), ("p90", 90), ("max", 100))},
         "slowest": [{"series": int(s), "end_us": float(end[s]), "fit_us": float(fit_us[s]),
                      "epi_us": float(epi_us[s]), "lbfgs_us": float(lb_us[s]),
                      "polish_us": float(pol_us[s]), "n_newton": int(nnewton[s]), "hessians": int(npe[s]), "hess_us": float(hess_us[s]), "sweep_us": float(sweep_us[s]),
                      "qp_us": float(qp_us[s]), "ls_us": float(ls_us[s]), "restore_us": float(rs_us[s]),
                      "n_eval": int(ne[s]), "status": int(st[s])}
                     for s in slow],
         "fit_us_vs_n_eval_corr": float(np.corrcoef(fit_us, ne)[0, 1]),
         "lbfgs_us_per_eval": {q: float(np.percentile(lb_us / np.maximum(ne, 1), p)) for q, p in
                               (("p10", 10), ("p50", 50), ("p90", 90))},
         "n_newton": {q: float(np.percentile(nnewton, p)) for q, p in
                      (("p50", 50), ("p90", 90), ("max", 100))},
         "hess_us_per_hessian_p50": float(np.median(hess_us / np.maximum(npe, 1))),
         "sweep_us_p50": float(np.median(sweep_us)),
         "polish_us_vs_newton_corr": float(np.corrcoef(pol_us, nnewton)[0, 1]),
         "hessians": {q: float(np.percentile(npe, p)) for q, p in
                      (("p50", 50), ("p90", 90), ("max", 100))},
         "polish_us_vs_hessians_corr": float(np.corrcoef(pol_us, npe)[0, 1]),
         "polish_us_p50_by_hessians": {int(h): float(np.median(pol_us[npe == h])) for h in np.unique(npe)},
         "by_block_half": {"blocks_lt_256_fit_p50": float(np.median(fit_us[:256])),
                           "blocks_ge_256_fit_p50": float(np.median(fit_us[256:]))}}
    res["runs"].append(r)
    print(json.dumps(r), flush=True)
if out_path:
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
