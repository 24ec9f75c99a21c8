"""Diagnostic: per-phase cycle shares of one series' evaluations (block 0).
Builds libprophet_hip_stamps.so (-DPF_STAMPS) and loads it instead of the product lib."""
import ctypes, os, subprocess, sys, time
import numpy as np, torch
sys.path.insert(0, ".")
here = "distributed-forecasting_amd"
out = os.environ.get("PF_STAMPS_LIB") or os.path.abspath("diag_exp/libprophet_hip_stamps.so")
if not os.path.exists(out):  # build here (CPU container), not on the GPU box
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                       "-DPF_STAMPS", "-Iinclude", f"-I{here}/csrc", "-o", out, f"{here}/csrc/pf_engine.hip"])
from distributed_forecasting_amd import _lib
_lib.load(os.path.abspath(out))
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ds = synthetic.daily_dates(); Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device="cuda"); Yd[:, :grid.T] = torch.from_numpy(Y).cuda()
lib = _lib._lib
buf = (ctypes.c_ulonglong * 32)()
lib.pf_debug_stamps(buf, 1)
for polish in (False,):
    torch.cuda.synchronize(); t0 = time.time()
    fit = eng.fit(grid, Yd, polish=polish); torch.cuda.synchronize(); dt = time.time() - t0
    lib.pf_debug_stamps(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    ne = fit.n_eval[0].item()
    ph = {"rows": v[2]-v[1], "wave reduce": v[3]-v[2], "barrier+assemble": v[4]-v[3],
          "lbfgs+publish+barrier": v[5]-v[4]}
    tot = sum(ph.values())
    print(f"polish={polish} fit {dt*1e3:.2f} ms; series0 n_eval={ne}; cycles/eval total {tot/ne:.0f}")
    for k_, c in ph.items():
        print(f"   {k_:22s} {c/ne:8.0f} cycles/eval  {100*c/tot:5.1f}%")
    print(f"   lbfgs_advance: state load {(v[7]-v[6])/ne:.0f}  step body {(v[8]-v[7])/ne:.0f} (per eval)")
    it = fit.n_iter[0].item()
    print(f"   LS_OK ({it} iters): fused-reduction {(v[11]-v[10])/it:.0f}  update+solve {(v[12]-v[11])/it:.0f} cycles/iter")
# polish phases (block 0, all Newton iterations of all polish passes)
torch.cuda.synchronize(); lib.pf_debug_stamps(buf, 1)
t0 = time.time(); fit = eng.fit(grid, Yd); torch.cuda.synchronize(); dt = time.time() - t0
lib.pf_debug_stamps(buf, 1)
v = np.array(list(buf), dtype=np.float64)
print(f"default fit {dt*1e3:.2f} ms; series0 n_eval={fit.n_eval[0].item()} status={fit.status[0].item()}")
nh = max(v[15], 1)
print(f"   polish: {v[15]:.0f} Hessians: total {(v[21]-v[20])/nh:.0f}/Hessian (H1 rows {(v[13]-v[20])/nh:.0f}, H2 MFMA {(v[14]-v[13])/nh:.0f}, H3+H4 {(v[21]-v[14])/nh:.0f}); initial sweeps {(v[24]-v[21]):.0f} total; qp {(v[22]-v[19]):.0f} total; line search {(v[17]-v[16]):.0f} total cycles")
print(f"   qp: initial sweeps {v[26]:.0f}  iterations {v[27]:.0f}  symv {(v[29]-v[28]):.0f}  rev-sweeps {(v[31]-v[30]):.0f} cycles; Newton steps (block 0) {v[18]:.0f}")
