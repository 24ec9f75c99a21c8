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


NS_PER_HOUR = 3_600_000_000_000


def hourly_dates(start="2017-01-01", n_hours: int = 8760) -> np.ndarray:
    """SURVEY.md §8d config 5 grid: ``start`` 00:00 + k hours."""
    s = np.datetime64(start, "D").astype("datetime64[ns]").astype(np.int64)
    return s + NS_PER_HOUR * np.arange(n_hours, dtype=np.int64)


def saturating_matrix(n_series: int, ds_ns: np.ndarray, seed: int = 20261015 + 4):
    """Config-5-shaped series for logistic growth: a saturating level
    C_s sigma(r_s (t - t0_s)) with yearly, weekly and (for sub-daily grids)
    daily multiplicative seasonality and noise.  Returns (Y, cap) with the
    constant capacity cap_s = 1.2 max(y_s)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    T = ds_ns.shape[0]
    d = (ds_ns / 1e9) / 86400.0
    t = np.arange(T) / max(T - 1, 1)
    C = np.exp(rng.uniform(np.log(20), np.log(200), n_series))
    r = rng.uniform(2.0, 8.0, n_series)
    t0 = rng.uniform(0.2, 0.7, n_series)
    ay = rng.uniform(0.05, 0.2, n_series)
    aw = rng.uniform(0.05, 0.15, n_series)
    ad = rng.uniform(0.0, 0.2, n_series)
    ph = rng.uniform(0, 2 * np.pi, (n_series, 3))
    lvl = C[:, None] / (1.0 + np.exp(-r[:, None] * (t[None, :] - t0[:, None])))
    seas = ((1 + ay[:, None] * np.sin(2 * np.pi * d[None, :] / 365.25 + ph[:, :1]))
            * (1 + aw[:, None] * np.sin(2 * np.pi * d[None, :] / 7.0 + ph[:, 1:2]))
            * (1 + ad[:, None] * np.sin(2 * np.pi * d[None, :] + ph[:, 2:3])))
    Y = np.maximum(0.0, lvl * seas + rng.normal(0.0, 1.0, (n_series, T)) * 0.05 * C[:, None])
    cap = np.repeat((1.2 * Y.max(axis=1))[:, None], T, axis=1)
    return Y, cap


def staggered_frame(n_stores: int = 10, n_items: int = 50, start="2013-01-01",
                    end="2017-12-31", n_starts: int = 50, max_delay_days: int = 730,
                    n_ends: int = 1, config_index: int = 1, seed: int = 20261017):
    """Store-item table with staggered launches: every series is generated on
    the full daily grid, then keeps the rows from its own launch date
    (one of ``n_starts`` dates spread over ``max_delay_days``) and, with
    ``n_ends`` > 1, stops at one of ``n_ends`` end dates in the last 60 days.
    A real store-item table's shape (new items, delisted items) instead of
    the Kaggle table's single shared grid (02_training.py:277-282)."""
    import pandas as pd
    ds = daily_dates(start, end)
    n = n_stores * n_items
    Y = sales_matrix(n, ds, config_index)
    rng = np.random.Generator(np.random.PCG64(seed))
    offs = np.linspace(0, max_delay_days, n_starts).astype(np.int64)
    first = offs[rng.integers(0, n_starts, n)]
    ends = np.linspace(0, 60 if n_ends > 1 else 0, n_ends).astype(np.int64)
    last = ds.shape[0] - ends[rng.integers(0, n_ends, n)]
    stores = np.repeat(np.arange(1, n_stores + 1), n_items)
    items = np.tile(np.arange(1, n_items + 1), n_stores)
    parts = []
    for s in range(n):
        sl = slice(int(first[s]), int(last[s]))
        m = sl.stop - sl.start
        parts.append(pd.DataFrame({
            "ds": ds[sl].astype("datetime64[ns]"),
            "store": np.full(m, stores[s], np.int32),
            "item": np.full(m, items[s], np.int32),
            "y": Y[s, sl],
        }))
    return pd.concat(parts, ignore_index=True)
