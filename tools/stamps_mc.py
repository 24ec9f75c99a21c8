"""Diagnostic: cycle split of k_predict_mc (block 0, wave 0): setup vs per-row
value generation vs order-statistic selection.  Uses the -DPF_STAMPS build."""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, ".")
from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath("diag_exp/libprophet_hip_stamps.so"))
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, batch as B
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
method = sys.argv[2] if len(sys.argv) > 2 else "exact"        # "sample": configs[3]'s literal loop
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 1              # 3: 730-day configs[3] shape
ds = synthetic.daily_dates() if cfg != 3 else synthetic.daily_dates("2016-01-01", "2017-12-30")
Y = synthetic.sales_matrix(n, ds, config_index=cfg)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
fit = eng.fit(grid, Yd)
fg = eng.predict_grid(fit, B.future_dates(ds, 90))
buf = (ctypes.c_ulonglong * 32)()
torch.cuda.synchronize(); _lib._lib.pf_debug_stamps(buf, 1)
eng.predict(fit, fg, seed=1, interval_method=method); torch.cuda.synchronize()
_lib._lib.pf_debug_stamps(buf, 1)
v = np.array(list(buf), dtype=np.float64)
rows = max(v[9], 1)
print(f"k_predict_mc block (0,0) wave 0: setup {v[1]-v[0]:.0f} cycles; {rows:.0f} rows; row prologue {v[2]-v[1]:.0f}; per row: "
      f"absorb {(v[4]-v[3])/rows:.0f}  normals {(v[5]-v[4])/rows:.0f}  trend samples + v {(v[6]-v[5])/rows:.0f}  select {(v[7]-v[6])/rows:.0f} cycles")
print(f"  select split per row: lane minima + threshold sort {(v[10]-v[6])/rows:.0f}, compaction {(v[11]-v[10])/rows:.0f}, "
      f"candidate sort {(v[12]-v[11])/rows:.0f}, ranks + lerp {(v[7]-v[12])/rows:.0f} cycles")
