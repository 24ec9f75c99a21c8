"""Diagnostic: host-side profile of the drop-in forecast_store_items call at
configs[1] (500 series x 1826 days, pandas in / out) on the GPU box."""
import cProfile
import pstats
import sys

sys.path.insert(0, ".")
import distributed_forecasting_amd as dfa  # noqa: E402
from distributed_forecasting_amd import synthetic  # noqa: E402

df = synthetic.store_item_frame(10, 50)
dfa.forecast_store_items(df)
dfa.forecast_store_items(df)
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    dfa.forecast_store_items(df)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
