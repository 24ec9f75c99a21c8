"""Drop-in host path at configs[1] (500 series x 1826 days, pandas in /
pandas out) on the GPU box: forecast_store_items (dense fast path and the
general grouping path on a row-shuffled copy), with cross-validation
metrics, and ForecastStoreItemModel.predict; then a cProfile of the fast
path.  Prints one JSON line and the profile."""
import cProfile
import json
import os
import pstats
import sys
import tempfile
import time

import numpy as np
import pandas as pd
import torch

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

df = synthetic.store_item_frame(10, 50)
n = 500
shuf = df.sample(frac=1.0, random_state=0).reset_index(drop=True)


def timed(fn, k=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k, r


res = {}
dt, fr = timed(lambda: dfa.forecast_store_items(df))
res["forecast_store_items"] = {"series_per_s": n / dt, "ms": dt * 1e3, "rows": len(fr)}
dt, fr2 = timed(lambda: dfa.forecast_store_items(shuf), 3)
res["forecast_store_items_general_path"] = {"series_per_s": n / dt, "ms": dt * 1e3}
a = fr.sort_values(["store", "item", "ds"]).reset_index(drop=True)
b = fr2.sort_values(["store", "item", "ds"]).reset_index(drop=True)
res["general_equals_fast"] = bool(all(np.array_equal(a[k].to_numpy(), b[k].to_numpy()) for k in ("ds", "store", "item", "yhat", "yhat_upper", "yhat_lower")))
dt, (fr3, met) = timed(lambda: dfa.forecast_store_items(df, cv_metrics=True, return_metrics=True), 3)
res["forecast_store_items_cv"] = {"series_per_s": n / dt, "ms": dt * 1e3,
                                  "mse_mean": float(met["mse"].mean()),
                                  "mape_mean": float(met["mape"].mean())}
with tempfile.TemporaryDirectory() as tmp:
    store = dfa.ParamsStore(os.path.join(tmp, "p"))
    dfa.forecast_store_items(df, params_store=store)
    model = dfa.ForecastStoreItemModel(store)
    futd = dfa.future_dates(synthetic.daily_dates(), 90)
    keys = np.stack(np.meshgrid(np.arange(1, 11), np.arange(1, 51), indexing="ij"), -1).reshape(-1, 2)
    inp = pd.DataFrame({"ds": np.tile(futd.astype("datetime64[ns]"), n),
                        "store": np.repeat(keys[:, 0], len(futd)).astype(np.int32),
                        "item": np.repeat(keys[:, 1], len(futd)).astype(np.int32)})
    dt, out = timed(lambda: model.predict(None, inp))
    res["pyfunc_predict"] = {"series_per_s": n / dt, "ms": dt * 1e3, "rows": len(out)}
    res["pyfunc_equals_fit_frame"] = bool(np.array_equal(out["yhat"].to_numpy(), fr["yhat"].to_numpy()))
print(json.dumps(res))
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    dfa.forecast_store_items(df)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
