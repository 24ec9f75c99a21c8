"""Diagnostic: where the exact-MAP polish spends its cycles (block 0 of each
launch; -DPF_STAMPS build), one series per launch.

    python tools/stamps_polish.py [config 1|4] [n_series]
Per series: Newton steps, sweeps, QP iterations, and cycles in the Hessian,
the sweep-in of the free set, the QP, and the Armijo evaluations."""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath(os.environ.get("PF_STAMPS_LIB", "diag_exp/libprophet_hip_stamps.so")))
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, holidays as H
from distributed_forecasting_amd.engine import ProphetConfig
cfgi = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cfg = ProphetConfig.reference()
hol, cap = None, None
if cfgi == 4:
    ds = synthetic.hourly_dates(n_hours=8760)
    Y, cap = synthetic.saturating_matrix(n, ds)
    cfg.growth = "logistic"
    seasons = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
    hol = H.holiday_spec(H.synthetic_holidays([2017, 2018]), cfg.holidays_prior_scale, cfg.seasonality_mode)
else:
    ds = synthetic.daily_dates()
    Y = synthetic.sales_matrix(n, ds)
    seasons = cfg.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
eng = dfa.Engine(0, cfg)
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=hol)
buf = (ctypes.c_ulonglong * 32)()
rows = []
for i in range(n):
    Yd = torch.zeros((1, grid.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :grid.T] = torch.from_numpy(Y[i:i + 1]).cuda()
    cd = None
    if cap is not None:
        cd = torch.zeros_like(Yd)
        cd[:, :grid.T] = torch.from_numpy(cap[i:i + 1]).cuda()
    torch.cuda.synchronize(); _lib._lib.pf_debug_stamps(buf, 1)
    eng.ctx.set_timing(True)
    fit = eng.fit(grid, Yd, cap=cd, tile_min_series=-1)
    torch.cuda.synchronize()
    kt = {k: v for k, v, _ in eng.ctx.read_timings()}
    eng.ctx.set_timing(False)
    _lib._lib.pf_debug_stamps(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    rows.append(dict(hessians=v[15], polish_calls=v[23], damped=v[28], warm_qp_fail=v[29], lag_reject=v[30], backtracked=v[31], newton=v[18], sweeps=v[26], qp_it=v[27], hess=v[21] - v[20], sweep_in=v[24] - v[21],
                     qp=v[22] - v[19], armijo=v[17] - v[16], n_eval=int(fit.n_eval[0]),
                     status=int(fit.status[0]), kernels={k: round(x, 3) for k, x in kt.items()}))
    print(rows[-1], flush=True)
m = {k: float(np.mean([r[k] for r in rows])) for k in ("hessians", "polish_calls", "damped", "warm_qp_fail", "lag_reject", "backtracked", "newton", "sweeps", "qp_it", "hess", "sweep_in", "qp", "armijo")}
print("mean", {k: round(x) for k, x in m.items()})
print("cycles per Hessian", round(sum(r["hess"] for r in rows) / max(1, sum(r["hessians"] for r in rows))))
