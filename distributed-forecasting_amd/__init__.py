"""MI355X-native batched Prophet fit + forecast engine.

Drop-in for the per-(store, item) Prophet path of rafaelvp-db/distributed-forecasting
(notebooks/prophet/02_training.py:150-319, model_wrapper.py:11-73).  The
arithmetic runs in hand-written HIP kernels for gfx950 (``csrc/``) behind the C
ABI in ``include/prophet_hip.h``; this package is the host side.
"""
from ._lib import EngineUnavailable, STATUS_NAMES  # noqa: F401
from .engine import (DeviceGrid, Engine, FitResult, ProphetConfig, build_grid,  # noqa: F401
                     future_dates, pad_rows)

__all__ = ["Engine", "ProphetConfig", "FitResult", "DeviceGrid", "build_grid", "future_dates",
           "pad_rows", "EngineUnavailable", "STATUS_NAMES"]
