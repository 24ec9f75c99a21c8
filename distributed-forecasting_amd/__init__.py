"""MI355X-native batched Prophet fit + forecast engine.

Drop-in for the per-(store, item) Prophet path of rafaelvp-db/distributed-forecasting
(notebooks/prophet/02_training.py:150-319, model_wrapper.py:11-73,
04_inference.py:4-16).  The arithmetic runs in hand-written HIP kernels for
gfx950 (``csrc/``) behind the C ABI in ``include/prophet_hip.h``; this package
is the host side.  There is no CPU fallback: without the built library every
entry point raises ``EngineUnavailable``.
"""
from ._lib import EngineUnavailable, STATUS_NAMES, CV_METRICS  # noqa: F401
from .engine import (DeviceGrid, Engine, FitResult, ProphetConfig, build_grid,  # noqa: F401
                     pad_rows)
from .batch import FittedBatch, bucket_groups, series_id, shard_of  # noqa: F401
from .forecaster import Prophet, SIMPLE_ATTRIBUTES  # noqa: F401
from .training import (train_model, make_prediction, forecast_item,  # noqa: F401
                       forecast_store_item, forecast_store_items, forecast_items,
                       extract_params, reference_model, allocate_forecasts,
                       forecast_partitions)
from .serving import ParamsStore, ForecastStoreItemModel, predict_udf, register_model  # noqa: F401
from .diagnostics import cv_metrics_batch, cv_metrics_device, generate_cutoffs  # noqa: F401
from .engine import future_dates  # noqa: F401
from .holidays import HolidaySpec, holiday_spec  # noqa: F401
from . import tuning  # noqa: F401
from .graphs import ForecastStep  # noqa: F401
from . import serialize  # noqa: F401
from .tuning import hyperparameter_search, sample_trials  # noqa: F401

__all__ = ["Engine", "ProphetConfig", "FitResult", "DeviceGrid", "build_grid", "future_dates",
           "pad_rows", "EngineUnavailable", "STATUS_NAMES", "CV_METRICS", "FittedBatch",
           "bucket_groups", "series_id", "shard_of", "Prophet", "SIMPLE_ATTRIBUTES",
           "train_model", "make_prediction", "forecast_item", "forecast_store_item",
           "forecast_store_items", "forecast_items", "extract_params", "reference_model",
           "ParamsStore", "ForecastStoreItemModel", "predict_udf", "register_model",
           "cv_metrics_batch", "cv_metrics_device", "generate_cutoffs", "allocate_forecasts",
           "forecast_partitions", "HolidaySpec", "holiday_spec", "tuning",
           "hyperparameter_search", "sample_trials", "ForecastStep"]
