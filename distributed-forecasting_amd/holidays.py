"""Holiday indicator columns (UPSTREAM Prophet 1.0 ``make_holiday_features`` /
``construct_holiday_dataframe``; SURVEY.md §8a row a2, configs[4]).

A holidays frame has columns ``holiday`` (name), ``ds`` (date) and optionally
``lower_window`` / ``upper_window`` (day offsets, default 0) and
``prior_scale`` (default ``holidays_prior_scale``).  Every (holiday, offset)
pair becomes one 0/1 column named ``f"{holiday}_delim_{+|-}{|offset|}"``, set
on every row whose calendar date is the holiday's date + offset (all 24 rows
of the day for hourly data), columns sorted by name — the same set at fit and
predict time, so the predict grid reuses the fit's columns.  The columns are
appended after the Fourier blocks and go to the device grid builder
(``pf_build_grid`` ``extra_cols``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import pandas as pd

NS_PER_DAY = 86_400 * 10**9


@dataclass(frozen=True)
class HolidaySpec:
    """Column layout derived from a holidays frame (hashable: cached vectors)."""
    names: tuple            # column names, sorted
    prior_scales: tuple     # per column
    holidays: tuple         # distinct holiday names (UPSTREAM train_holiday_names)
    rows: tuple             # (column index, day number) pairs that are set
    mode: str               # 'multiplicative' | 'additive' (UPSTREAM holidays_mode)

    @property
    def n(self) -> int:
        return len(self.names)


def _day(ns) -> np.ndarray:
    return np.floor_divide(np.asarray(ns, np.int64), NS_PER_DAY)


def holiday_spec(holidays: pd.DataFrame, holidays_prior_scale: float = 10.0,
                 mode: str = "multiplicative") -> HolidaySpec:
    """UPSTREAM make_holiday_features' column bookkeeping (names, prior scales,
    conflicting-prior check) for a holidays frame."""
    if holidays is None or len(holidays) == 0:
        return HolidaySpec((), (), (), (), mode)
    if "holiday" not in holidays or "ds" not in holidays:
        raise ValueError('holidays must be a DataFrame with "holiday" and "ds" columns.')
    hd = holidays.copy()
    hd["ds"] = pd.to_datetime(hd["ds"])
    if hd["ds"].isnull().any():
        raise ValueError("Found a NaN in holidays dataframe.")
    has_lw, has_uw = "lower_window" in hd, "upper_window" in hd
    if has_lw != has_uw:
        raise ValueError("Holidays must have both lower_window and upper_window, or neither")
    prior = {}
    cols = {}
    for row in hd.itertuples(index=False):
        try:
            lw = int(getattr(row, "lower_window", 0))
            uw = int(getattr(row, "upper_window", 0))
        except ValueError:
            lw, uw = 0, 0
        if lw > 0 or uw < 0:
            raise ValueError("Holiday lower_window should be <= 0 and upper_window should be >= 0")
        ps = float(getattr(row, "prior_scale", holidays_prior_scale))
        if np.isnan(ps):
            ps = float(holidays_prior_scale)
        if ps <= 0:
            raise ValueError("Prior scale must be > 0")
        name = str(row.holiday)
        if name in prior and prior[name] != ps:
            raise ValueError(f"Holiday {name!r} does not have consistent prior scale specification.")
        prior[name] = ps
        d0 = int(_day(pd.Timestamp(row.ds).normalize().value))
        for off in range(lw, uw + 1):
            key = "{}_delim_{}{}".format(name, "+" if off >= 0 else "-", abs(off))
            cols.setdefault(key, set()).add(d0 + off)
    names = tuple(sorted(cols))
    rows = tuple((j, d) for j, k in enumerate(names) for d in sorted(cols[k]))
    return HolidaySpec(names, tuple(prior[k.split("_delim_")[0]] for k in names),
                       tuple(prior), rows, mode)


def holiday_columns(spec: HolidaySpec, ds_ns) -> np.ndarray:
    """[n_columns, T] float64 indicators on the dates ``ds_ns``."""
    days = _day(ds_ns)
    X = np.zeros((spec.n, days.shape[0]), np.float64)
    for j, d in spec.rows:
        X[j, days == d] = 1.0
    return X


def synthetic_holidays(years, n_per_year: int = 10, seed: int = 20261019) -> pd.DataFrame:
    """configs[4]: ``n_per_year`` holidays per year, window [0, 0] — fixed
    day-of-year per holiday name (like calendar holidays), drawn once."""
    rng = np.random.default_rng(seed)
    doy = np.sort(rng.choice(np.arange(1, 366), size=n_per_year, replace=False))
    rows = []
    for y in years:
        for h, d in enumerate(doy):
            rows.append((f"hol{h:02d}", pd.Timestamp(year=int(y), month=1, day=1) + pd.Timedelta(days=int(d) - 1)))
    return pd.DataFrame(rows, columns=["holiday", "ds"]).assign(lower_window=0, upper_window=0)
