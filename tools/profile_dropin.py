"""Host profile of the drop-in surfaces at the headline's shape (500 x 1826
days, 90-day horizon): forecast_store_items(df) and
ForecastStoreItemModel.predict under cProfile, plus the wall time per call.
    python tools/profile_dropin.py [calls] [out.txt]"""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pandas as pd
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import synthetic

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
out_path = sys.argv[2] if len(sys.argv) > 2 else None
ds = synthetic.daily_dates()
n, T = 500, len(ds)
Y = synthetic.sales_matrix(n, ds, config_index=1)
keys = np.stack([np.repeat(np.arange(1, 11), 50), np.tile(np.arange(1, 51), 10)], 1)
df = pd.DataFrame({"ds": np.tile(ds.astype("datetime64[ns]"), n),
                   "store": np.repeat(keys[:, 0], T).astype(np.int32),
                   "item": np.repeat(keys[:, 1], T).astype(np.int32),
                   "y": Y.reshape(-1)})
buf = io.StringIO()


def run(name, fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / calls * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    pr.disable()
    buf.write(f"==== {name}: {ms:.3f} ms/call ({n / ms * 1e3:.0f} series/s)\n")
    st = pstats.Stats(pr, stream=buf)
    st.sort_stats("tottime").print_stats(25)
    print(f"{name}: {ms:.3f} ms/call", flush=True)


run("forecast_store_items", lambda: dfa.forecast_store_items(df))
os.environ["PF_NO_FUSE"] = "1"      # A/B: pf_fit_forecast runs the separate launches
run("forecast_store_items (fuse off)", lambda: dfa.forecast_store_items(df))
del os.environ["PF_NO_FUSE"]
with tempfile.TemporaryDirectory() as tmp:
    store = dfa.ParamsStore(os.path.join(tmp, "params"), writer="r0")
    dfa.forecast_store_items(df, params_store=store)
    model = dfa.ForecastStoreItemModel(store)
    futd = dfa.future_dates(ds, 90)
    inp = pd.DataFrame({"ds": np.tile(futd.astype("datetime64[ns]"), n),
                        "store": np.repeat(keys[:, 0], len(futd)).astype(np.int32),
                        "item": np.repeat(keys[:, 1], len(futd)).astype(np.int32)})
    run("pyfunc_predict", lambda: model.predict(None, inp))
text = buf.getvalue()
if out_path:
    with open(out_path, "w") as fh:
        fh.write(text)
else:
    print(text)
