"""Dev tool: back-to-back replays of one captured ForecastStep vs two
captured steps (two graph execs of the same batch shape) alternated on the
same stream — is the inter-replay gap the graph launch waiting on the
previous instance of the same graph?"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic, batch as B
n = 500
ds = synthetic.daily_dates()
Y = synthetic.sales_matrix(n, ds)
eng = dfa.Engine(0)
sid = torch.arange(n, dtype=torch.int32, device="cuda")
steps = [dfa.ForecastStep(eng, ds, n, horizon=90, series_id=sid) for _ in range(2)]
for s in steps:
    s.set_inputs(Y)
    s.run()
    s.capture()
torch.cuda.synchronize()
K = 40
for trial in range(3):
    for mode in ("one", "two"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            (steps[0] if mode == "one" else steps[k & 1]).replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"{mode}: {el / K * 1e3:.4f} ms/step  {n * K / el:.0f} series/s", flush=True)
