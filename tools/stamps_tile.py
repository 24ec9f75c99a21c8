"""Diagnostic: per-phase cycles per evaluation of the tiled fit kernel K3T
(block 0, wave 0 lane 0 s_memtime sums; -DPF_STAMPS build, never the product).
    python tools/stamps_tile.py [n]"""
import ctypes, os, subprocess, sys, time
import numpy as np, torch
sys.path.insert(0, ".")
here = "distributed-forecasting_amd"
out = os.environ.get("PF_STAMPS_LIB") or os.path.abspath("diag_exp/libprophet_hip_stamps.so")
if not os.path.exists(out):
    subprocess.check_call(["sh", "tools/build_stamps.sh"])
from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath(out))
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
c4 = len(sys.argv) > 2 and sys.argv[2] == "c4"     # configs[4]: hourly logistic, P = 72
cap = None
if c4:
    from distributed_forecasting_amd import holidays as H
    from distributed_forecasting_amd.engine import ProphetConfig
    cfg = ProphetConfig.reference()
    cfg.growth = "logistic"
    ds = synthetic.hourly_dates(n_hours=8760)
    Y, cp = synthetic.saturating_matrix(n, ds)
    eng = dfa.Engine(0, cfg)
    seasons = [("yearly", 365.25, 10), ("weekly", 7.0, 3), ("daily", 1.0, 4)]
    hol = H.holiday_spec(H.synthetic_holidays([2017, 2018]), 10.0)
    grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), holidays=hol)
    cap = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); cap[:, :grid.T] = torch.from_numpy(cp).cuda()
else:
    ds = synthetic.daily_dates(); Y = synthetic.sales_matrix(n, ds, config_index=2)
    eng = dfa.Engine(0)
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
lib = _lib._lib
buf = (ctypes.c_ulonglong * 32)()
eng.fit(grid, Yd, cap=cap, polish=False, tile_min_series=1); torch.cuda.synchronize()
lib.pf_debug_stamps(buf, 1)
t0 = time.time()
fit = eng.fit(grid, Yd, cap=cap, polish=False, tile_min_series=1, lbfgs_warmup=0); torch.cuda.synchronize()
dt = time.time() - t0
lib.pf_debug_stamps(buf, 1)
v = np.array(list(buf), dtype=np.float64)
ne = max(v[7], 1)
ph = {"row pass (wave 0)": v[1] - v[0], "barrier wait": v[2] - v[1], "assemble": v[3] - v[2],
      "barrier+zero+lbfgs": v[4] - v[3], "publish": v[5] - v[4], "end barrier": v[6] - v[5]}
print(f"n={n} fit(polish=False) {dt*1e3:.1f} ms; tile 0: {ne:.0f} evaluations; "
      f"series0 n_eval={fit.n_eval[0].item()}")
tot = sum(ph.values())
for k, c in ph.items():
    print(f"   {k:20s} {c / ne:9.0f} cycles/eval {100 * c / tot:5.1f}%")
