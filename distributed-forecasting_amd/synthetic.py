"""Synthetic Kaggle store-item-shaped daily sales.

y = max(0, round(L (1 + g t) (1 + a sin(2π d/365.25 + φ)) w[dow] + ε))
L ~ LogUniform(10, 100), g ~ U(0, 0.5), a ~ U(0.1, 0.4),
w[dow] = 1 + 0.15 U(-1, 1) normalised to mean 1, ε ~ N(0, (0.1 L)^2);
integer sales like the reference's ``sales int`` schema (02_training.py:33).
Base seed 20261015 + config index (numpy PCG64).
"""
from __future__ import annotations

import numpy as np

NS_PER_DAY = 86400 * 10**9
BASE_SEED = 20261015


def daily_dates(start="2013-01-01", end="2017-12-31") -> np.ndarray:
    s = np.datetime64(start, "D").astype("datetime64[ns]").astype(np.int64)
    e = np.datetime64(end, "D").astype("datetime64[ns]").astype(np.int64)
    return np.arange(s, e + NS_PER_DAY, NS_PER_DAY, dtype=np.int64)


def sales_matrix(n_series: int, ds_ns: np.ndarray, config_index: int = 1,
                 seed: int | None = None) -> np.ndarray:
    """[n_series, T] float64 integer-valued sales on the grid ``ds_ns``."""
    rng = np.random.Generator(np.random.PCG64(BASE_SEED + config_index if seed is None else seed))
    T = ds_ns.shape[0]
    d = (ds_ns / 1e9) / 86400.0
    t = np.arange(T) / max(T - 1, 1)
    L = np.exp(rng.uniform(np.log(10), np.log(100), n_series))
    g = rng.uniform(0, 0.5, n_series)
    a = rng.uniform(0.1, 0.4, n_series)
    ph = rng.uniform(0, 2 * np.pi, n_series)
    w = 1 + 0.15 * rng.uniform(-1, 1, (n_series, 7))
    w /= w.mean(axis=1, keepdims=True)
    dow = (np.floor(d).astype(np.int64) + 3) % 7     # 1970-01-01 was a Thursday
    base = (L[:, None] * (1 + g[:, None] * t[None, :])
            * (1 + a[:, None] * np.sin(2 * np.pi * d[None, :] / 365.25 + ph[:, None]))
            * w[:, dow])
    eps = rng.normal(0.0, 1.0, (n_series, T)) * (0.1 * L[:, None])
    return np.maximum(0.0, np.round(base + eps))


def store_item_frame(n_stores: int = 10, n_items: int = 50, start="2013-01-01",
                     end="2017-12-31", config_index: int = 1):
    """Long-format frame like hackathon.sales.raw: (ds, store, item, y)."""
    import pandas as pd
    ds = daily_dates(start, end)
    Y = sales_matrix(n_stores * n_items, ds, config_index)
    stores = np.repeat(np.arange(1, n_stores + 1), n_items)
    items = np.tile(np.arange(1, n_items + 1), n_stores)
    T = ds.shape[0]
    return pd.DataFrame({
        "ds": np.tile(ds.astype("datetime64[ns]"), n_stores * n_items),
        "store": np.repeat(stores, T).astype(np.int32),
        "item": np.repeat(items, T).astype(np.int32),
        "y": Y.reshape(-1),
    })
