"""Diagnostic: which path K5's order-statistic selection takes per row
(wave_tail_select): the moment threshold (step 1), the lane-minima
threshold (step 2), the bisection fallback — counted over every wave of
the fused forecast epilogue (-DPF_STAMPS build, reference layout unit).
    python tools/select_paths.py [n] [config_index]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath("diag_exp/libprophet_hip_stamps.so"))
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds, config_index=cfg)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
Yd[:, :g.T] = torch.from_numpy(Y).cuda()
fg = dfa.build_grid(dfa.future_dates(ds, 90), seasons, start_ns=g.start_ns, t_scale_ns=g.t_scale_ns,
                    t_change=g.t_change)
buf = (ctypes.c_ulonglong * 32)()
torch.cuda.synchronize()
_lib._lib.pf_debug_stamps(buf, 1)
fit, out, met, fused = eng.fit_forecast(g, Yd, fg, components=False, metrics="fast")
torch.cuda.synchronize()
_lib._lib.pf_debug_stamps(buf, 1)
v = np.array(list(buf), dtype=np.float64)
rows = max(v[14], 1)
print(f"fused={fused} selections {v[14]:.0f}: step 1 (moment threshold) {v[13] / rows:.3f}, "
      f"step 2 {1 - v[13] / rows:.3f}, bisection (per tail) {v[25] / rows:.3f}")
