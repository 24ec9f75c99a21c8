"""Device-level batched Prophet engine (HIP kernels via the C ABI).

This is the layer the drop-in API (forecaster.py / training.py) and bench.py
sit on.  Inputs and outputs are torch tensors resident on the GPU; torch is
only used for device memory and the stream handle.  Every compute step is one
of the HIP kernels behind include/prophet_hip.h — there is no CPU path.

Mapping to the reference:
  build_grid      → UPSTREAM setup_dataframe / make_all_seasonality_features /
                    set_changepoints (02_training.py:172 ``model.fit``)
  Engine.fit      → PyStan optimizing(LBFGS) on prophet.stan (02_training.py:172)
  Engine.predict  → make_future_dataframe + predict (02_training.py:201-205,
                    model_wrapper.py:58-61)
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib as L
from .holidays import HolidaySpec, holiday_columns

NS_PER_DAY = 86400 * 10**9
FIT_MODES = ("map", "stan_map", "stan")


def pad_rows(T: int) -> int:
    return ((int(T) + 127) // 128) * 128


# ---------------------------------------------------------------------------
# Prophet configuration (the reference's constructor, 02_training.py:162-169)
# ---------------------------------------------------------------------------
@dataclass
class ProphetConfig:
    growth: str = "linear"
    n_changepoints: int = 25
    changepoint_range: float = 0.8
    yearly_seasonality: object = "auto"
    weekly_seasonality: object = "auto"
    daily_seasonality: object = "auto"
    seasonality_mode: str = "additive"
    seasonality_prior_scale: float = 10.0
    holidays_prior_scale: float = 10.0
    changepoint_prior_scale: float = 0.05
    interval_width: float = 0.80
    uncertainty_samples: int = 1000
    # engine option (no Prophet counterpart): how deterministic-trend rows get
    # their interval endpoints — "exact" order statistics of the N draws (same
    # distribution, O(1) per row) or "sample" (materialise all N draws)
    interval_method: str = "exact"
    # engine option: which optimum the fit returns (PyStan optimizing() at
    # 02_training.py:172 stops where Stan's L-BFGS termination tests fire —
    # 1e-6..2e-4 relative short of the MAP at the |delta| kink, at a point
    # that moves with floating-point rounding):
    #   "map"      Stan L-BFGS warm-up handed to the certified exact-MAP
    #              polish (default; logistic growth runs Stan's full L-BFGS
    #              first, see Engine.fit_opts);
    #   "stan_map" Stan's full L-BFGS termination rules, then the polish (the
    #              same certified MAP, reached from Stan's endpoint);
    #   "stan"     Stan's full L-BFGS only: the reference-shaped answer
    #              (status = Stan's termination code, no certificate).
    fit_mode: str = "map"

    def __post_init__(self):
        if self.fit_mode not in FIT_MODES:
            raise ValueError(f"fit_mode must be one of {FIT_MODES}")

    @classmethod
    def reference(cls) -> "ProphetConfig":
        """Exactly the arguments of notebooks/prophet/02_training.py:162-169."""
        return cls(interval_width=0.95, growth="linear", daily_seasonality=False,
                   weekly_seasonality=True, yearly_seasonality=True,
                   seasonality_mode="multiplicative")

    # UPSTREAM parse_seasonality_args / set_auto_seasonalities
    @staticmethod
    def _order(arg, auto_disable, default):
        if arg == "auto":
            return 0 if auto_disable else default
        if arg is True:
            return default
        if arg is False or arg is None:
            return 0
        return int(arg)

    def seasons(self, first_ns: int, last_ns: int, min_dt_ns: int):
        span = last_ns - first_ns
        out = []
        yo = self._order(self.yearly_seasonality, span < 730 * NS_PER_DAY, 10)
        if yo > 0:
            out.append(("yearly", 365.25, yo))
        wo = self._order(self.weekly_seasonality,
                         span < 14 * NS_PER_DAY or min_dt_ns >= 7 * NS_PER_DAY, 3)
        if wo > 0:
            out.append(("weekly", 7.0, wo))
        do = self._order(self.daily_seasonality,
                         span < 2 * NS_PER_DAY or min_dt_ns >= NS_PER_DAY, 4)
        if do > 0:
            out.append(("daily", 1.0, do))
        return out


# ---------------------------------------------------------------------------
# context (one per device)
# ---------------------------------------------------------------------------
class Context:
    """One pf_ctx (its fit workspace and timing events).  ``close()`` (or
    garbage collection) calls pf_ctx_destroy; the per-device shared contexts
    of ``get`` live for the process."""
    _by_device: dict = {}

    def __init__(self, device: int):
        self.lib = L.load()
        self.device = device
        h = ctypes.c_void_p()
        rc = self.lib.pf_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"pf_ctx_create failed: {self.lib.pf_last_error(None).decode()}")
        self.h = h
        self._fin = weakref.finalize(self, Context._destroy, self.lib, h.value)
        self._fin.atexit = False       # process teardown releases the device anyway

    @staticmethod
    def _destroy(lib, handle):
        lib.pf_ctx_destroy(ctypes.c_void_p(handle))

    @property
    def closed(self) -> bool:
        return not self._fin.alive

    def close(self) -> None:
        """Destroy the C context now (hipFree of its workspace).  Callers must
        not have work in flight that uses it (graphs replaying it, launches on
        other streams): synchronise first.  The shared per-device contexts are
        never closed this way."""
        if Context._by_device.get(self.device) is self:
            raise RuntimeError("the shared per-device context is not closed by callers")
        if self._fin.alive:
            self._fin()
        self.h = ctypes.c_void_p(0)

    @classmethod
    def get(cls, device: int) -> "Context":
        if device not in cls._by_device:
            cls._by_device[device] = Context(device)
        return cls._by_device[device]

    def check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {self.lib.pf_last_error(self.h).decode()}")

    def set_timing(self, enable: bool):
        self.check(self.lib.pf_set_timing(self.h, 1 if enable else 0), "pf_set_timing")

    def read_timings(self):
        """[(kernel name, ms, workgroups)] for launches since the last read
        (HIP events recorded on each launch's stream; synchronises)."""
        buf = (L.PfKernelTime * 1024)()
        n = self.lib.pf_read_timings(self.h, buf, 1024)
        if n < 0:
            self.check(n, "pf_read_timings")
        return [(buf[i].name.decode(), float(buf[i].ms), int(buf[i].grid)) for i in range(n)]


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# ---------------------------------------------------------------------------
# K1: device grid
# ---------------------------------------------------------------------------
@dataclass
class DeviceGrid:
    ds_ns: np.ndarray              # host copy of the grid dates (sorted)
    start_ns: int
    t_scale_ns: int
    seasons: list                  # [(name, period, order)]
    T: int
    T_pad: int
    K: int
    S: int
    t: torch.Tensor
    XT: torch.Tensor
    t_change: torch.Tensor
    seg: torch.Tensor
    cp_first: torch.Tensor
    cp_idx: torch.Tensor | None = None
    n_changepoints_placed: int = 0
    holidays: HolidaySpec | None = None   # extra 0/1 columns after the Fourier blocks

    def as_pf(self) -> L.PfGrid:
        return L.PfGrid(self.T, self.T_pad, self.K, self.S, self.t.data_ptr(), self.XT.data_ptr(),
                        self.t_change.data_ptr(), self.seg.data_ptr(), self.cp_first.data_ptr())

    @property
    def fourier_orders(self):
        o = [0, 0, 0]
        for i, (_, _, order) in enumerate(self.seasons[:3]):
            o[i] = order
        return o


def _device_dates(ds_ns: np.ndarray, dev) -> torch.Tensor:
    """Grid dates on the device.  A regular grid (every daily / hourly bucket
    in practice) is generated there (start + k * step: an asynchronous device
    op), so building a grid never waits on a pageable host-to-device copy —
    which is stream-ordered and would stall the host until the GPU drained the
    previous batch's kernels."""
    T = ds_ns.shape[0]
    if T >= 2:
        step = int(ds_ns[1] - ds_ns[0])
        if step > 0 and int(ds_ns[-1] - ds_ns[0]) == step * (T - 1) and np.all(np.diff(ds_ns) == step):
            # one kernel: exact int64 arithmetic, start + k * step
            return torch.arange(int(ds_ns[0]), int(ds_ns[0]) + step * T, step, dtype=torch.int64,
                                device=dev)
    return _to_device_async(ds_ns, dev)


def build_grid(ds_ns: np.ndarray, seasons, *, start_ns: int, t_scale_ns: int,
               n_changepoints: int = 25, changepoint_range: float = 0.8,
               t_change: torch.Tensor | None = None, device: int = 0,
               holidays: HolidaySpec | None = None, T_pad: int | None = None) -> DeviceGrid:
    """Design grid on the GPU (K1).  With ``t_change=None`` the changepoints are
    placed (fit grid); otherwise they are reused (predict grid).  ``holidays``
    appends its indicator columns after the Fourier blocks (UPSTREAM
    make_all_seasonality_features order).  ``T_pad`` overrides the row stride
    (the sub-grids of a ragged batch share the largest one)."""
    ctx = Context.get(device)
    ds_ns = np.ascontiguousarray(np.asarray(ds_ns, dtype=np.int64))
    T = int(ds_ns.shape[0])
    Tp = pad_rows(T) if T_pad is None else int(T_pad)
    if Tp < T or Tp % 128:
        raise ValueError(f"T_pad={Tp} must be a multiple of 128 and >= T={T}")
    K = sum(2 * o for _, _, o in seasons)
    n_extra = holidays.n if holidays is not None else 0
    K += n_extra
    if K == 0:
        raise ValueError("no seasonality columns: the zero-feature dummy X is not supported yet")
    dev = torch.device("cuda", device)
    ds_d = _device_dates(ds_ns, dev)
    t = torch.empty(Tp, dtype=torch.float64, device=dev)
    XT = torch.empty(K * Tp, dtype=torch.float64, device=dev)
    seg = torch.empty(Tp, dtype=torch.int32, device=dev)
    sp = (L.PfSeason * max(1, len(seasons)))()
    for i, (_, period, order) in enumerate(seasons):
        sp[i].period = float(period)
        sp[i].order = int(order)
    if t_change is None:
        S_eff = L.num_changepoints(T, n_changepoints, changepoint_range)
        S = max(S_eff, 1)
        tc = torch.empty(S, dtype=torch.float64, device=dev)
        cp_idx = torch.empty(S, dtype=torch.int32, device=dev)
        ncp = n_changepoints
    else:
        tc = t_change
        S = int(tc.numel())
        cp_idx = None
        ncp = -1
        S_eff = S
    cp_first = torch.empty(S, dtype=torch.int32, device=dev)
    extra = None
    if n_extra:
        extra = _to_device_async(holiday_columns(holidays, ds_ns), dev)
    rc = ctx.lib.pf_build_grid(ctx.h, _ptr(ds_d), T, Tp, int(start_ns), int(t_scale_ns), sp,
                               len(seasons), _ptr(extra), n_extra, ncp, float(changepoint_range), _ptr(t),
                               _ptr(XT), _ptr(tc), _ptr(cp_idx), _ptr(seg), _ptr(cp_first), S,
                               _stream(device))
    ctx.check(rc, "pf_build_grid")
    return DeviceGrid(ds_ns, int(start_ns), int(t_scale_ns), list(seasons), T, Tp, K, S, t, XT,
                      tc, seg, cp_first, cp_idx, S_eff, holidays if n_extra else None)


def _to_device_async(a: np.ndarray, dev) -> torch.Tensor:
    """Host array -> device through a pinned staging copy (torch's caching host
    allocator keeps it until the copy ran): no stream-ordered pageable stall.
    (A 4-thread staging copy of the 7.3 MB headline y measured slower than
    torch's single copy on the box: 2.93 vs 2.72 ms per drop-in call,
    profiles/r04zf_dropin_host_profile.txt.)"""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dev.type == "cuda":
        t = t.pin_memory()
    return t.to(dev, non_blocking=True)


class RaggedGrid:
    """Series with different date grids in one launch (SURVEY §8a row a0 without
    one bucket per distinct date set).  Sub-grid g shares T_pad, K, S, the
    seasonality layout and the holiday spec with the others; series s uses
    ``grids[grid_of[s]]`` (the kernels bind it per workgroup, pf_problem.grids).
    Duck-types DeviceGrid for the engine: T is the envelope (max rows).

    Two constructions: ``RaggedGrid(list_of_DeviceGrid, grid_of)`` (any grids,
    e.g. with holiday columns) or ``RaggedGrid.build(...)`` — every sub-grid
    in three launches (pf_build_grids) into packed [G, ...] buffers."""

    def __init__(self, grids, grid_of: np.ndarray, device: int = 0):
        g0 = grids[0]
        for g in grids[1:]:
            if (g.T_pad, g.K, g.S, tuple(g.seasons)) != (g0.T_pad, g0.K, g0.S, tuple(g0.seasons)) \
                    or g.holidays != g0.holidays:
                raise ValueError("ragged sub-grids must share T_pad, K, S, seasonalities and holidays")
        self._grids = list(grids)
        self.G = len(grids)
        self.T_pad, self.K, self.S = g0.T_pad, g0.K, g0.S
        self.seasons, self.holidays = list(g0.seasons), g0.holidays
        self.Ts = np.asarray([g.T for g in grids], np.int64)
        self.T = int(self.Ts.max())
        self.packed = None
        self.device = device
        self._set_grid_of(grid_of, device)
        arr = (L.PfGrid * self.G)(*[g.as_pf() for g in grids])
        self.table = _to_device_async(np.frombuffer(bytes(arr), np.uint8).copy(),
                                      torch.device("cuda", device))

    def _set_grid_of(self, grid_of, device):
        gi = np.ascontiguousarray(np.asarray(grid_of, np.int32))
        if gi.size and (gi.min() < 0 or gi.max() >= self.G):
            raise ValueError("grid_of index out of range")
        self.grid_of_host = gi
        self.grid_of = _to_device_async(gi, torch.device("cuda", device))

    @classmethod
    def build(cls, ds_list, seasons, starts, scales, grid_of, *, device: int = 0,
              T_pad: int | None = None, n_changepoints: int = 25,
              changepoint_range: float = 0.8, t_change: torch.Tensor | None = None) -> "RaggedGrid":
        """All sub-grids on the device in three launches (pf_build_grids).
        ``ds_list[g]``: sorted dates of grid g; ``starts`` / ``scales``: its
        UPSTREAM start / t_scale (ns).  ``t_change`` ([G, S], a fit grid's
        packed changepoints): build forecast grids on them instead of placing
        changepoints."""
        ctx = Context.get(device)
        dev = torch.device("cuda", device)
        self = cls.__new__(cls)
        G = len(ds_list)
        Ts = np.asarray([len(d) for d in ds_list], np.int64)
        Tmax = int(Ts.max())
        Tp = pad_rows(Tmax) if T_pad is None else int(T_pad)
        if Tp < Tmax or Tp % 128:
            raise ValueError(f"T_pad={Tp} must be a multiple of 128 and >= {Tmax}")
        K = sum(2 * o for _, _, o in seasons)
        if K == 0:
            raise ValueError("no seasonality columns")
        if t_change is None:
            s_eff = {L.num_changepoints(int(T), n_changepoints, changepoint_range) for T in Ts}
            if len(s_eff) != 1:
                raise ValueError("ragged sub-grids must place the same number of changepoints")
            S_eff = s_eff.pop()
            S = max(S_eff, 1)
        else:
            S = S_eff = int(t_change.shape[1])
        prm = np.zeros((G, 6), np.int64)
        irregular, off = [], 0
        for g, d in enumerate(ds_list):
            d = np.asarray(d, np.int64)
            T = d.shape[0]
            step = int(d[1] - d[0]) if T >= 2 else 0
            regular = step > 0 and int(d[-1] - d[0]) == step * (T - 1) and bool(np.all(np.diff(d) == step))
            prm[g] = (off, T, int(starts[g]), int(scales[g]), int(d[0]), step if regular else 0)
            if not regular:
                irregular.append(d)
                off += T
        buf = np.concatenate([prm.ravel()] + irregular) if irregular else prm.ravel()
        bd = _to_device_async(buf, dev)
        t = torch.empty((G, Tp), dtype=torch.float64, device=dev)
        XT = torch.empty((G, K * Tp), dtype=torch.float64, device=dev)
        if t_change is None:
            tc = torch.empty((G, S), dtype=torch.float64, device=dev)
            cp_idx = torch.empty((G, S), dtype=torch.int32, device=dev)
            ncp = n_changepoints
        else:
            assert t_change.dtype == torch.float64 and t_change.shape[0] == G and t_change.is_contiguous()
            tc, cp_idx, ncp = t_change, None, -1
        seg = torch.empty((G, Tp), dtype=torch.int32, device=dev)
        cp_first = torch.empty((G, S), dtype=torch.int32, device=dev)
        table = torch.empty(G * ctypes.sizeof(L.PfGrid), dtype=torch.uint8, device=dev)
        sp = (L.PfSeason * max(1, len(seasons)))()
        for i, (_, period, order) in enumerate(seasons):
            sp[i].period = float(period)
            sp[i].order = int(order)
        rc = ctx.lib.pf_build_grids(ctx.h, G, _ptr(bd), ctypes.c_void_p(bd.data_ptr() + 8 * G * 6),
                                    Tmax, Tp, sp, len(seasons), ncp, float(changepoint_range),
                                    _ptr(t), _ptr(XT), _ptr(tc), _ptr(cp_idx), _ptr(seg),
                                    _ptr(cp_first), S, _ptr(table), _stream(device))
        ctx.check(rc, "pf_build_grids")
        self._grids = None
        self.G, self.T_pad, self.K, self.S, self.T = G, Tp, K, S, Tmax
        self.seasons, self.holidays = list(seasons), None
        self.Ts = Ts
        self.table = table
        self.packed = dict(ds=[np.asarray(d, np.int64) for d in ds_list],
                           starts=np.asarray(starts, np.int64), scales=np.asarray(scales, np.int64),
                           t=t, XT=XT, t_change=tc, cp_idx=cp_idx, seg=seg, cp_first=cp_first,
                           S_eff=S_eff, params=bd)
        self.device = device
        self._set_grid_of(grid_of, device)
        return self

    @property
    def grids(self):
        """Sub-grids as DeviceGrids (views into the packed buffers when built)."""
        if self._grids is None:
            p = self.packed
            self._grids = [
                DeviceGrid(p["ds"][g], int(p["starts"][g]), int(p["scales"][g]), list(self.seasons),
                           int(self.Ts[g]), self.T_pad, self.K, self.S, p["t"][g], p["XT"][g],
                           p["t_change"][g], p["seg"][g], p["cp_first"][g],
                           p["cp_idx"][g] if p["cp_idx"] is not None else None, p["S_eff"], None)
                for g in range(self.G)]
        return self._grids

    @property
    def n_grids(self) -> int:
        return self.G

    @property
    def fourier_orders(self):
        o = [0, 0, 0]
        for i, (_, _, order) in enumerate(self.seasons[:3]):
            o[i] = order
        return o

    @property
    def T_of(self) -> np.ndarray:
        """Rows of each series' own grid."""
        return self.Ts[self.grid_of_host]

    def as_pf(self) -> L.PfGrid:
        if self.packed is not None:
            p = self.packed
            return L.PfGrid(self.T, self.T_pad, self.K, self.S, p["t"].data_ptr(), p["XT"].data_ptr(),
                            p["t_change"].data_ptr(), p["seg"].data_ptr(), p["cp_first"].data_ptr())
        g0 = self._grids[0]
        return L.PfGrid(self.T, self.T_pad, self.K, self.S, g0.t.data_ptr(), g0.XT.data_ptr(),
                        g0.t_change.data_ptr(), g0.seg.data_ptr(), g0.cp_first.data_ptr())

    def tensors(self):
        out = [self.grid_of, self.table]
        if self.packed is not None:
            p = self.packed
            return out + [p["t"], p["XT"], p["t_change"], p["seg"], p["cp_first"], p["params"]]
        for g in self._grids:
            out += [g.t, g.XT, g.t_change, g.seg, g.cp_first]
        return out


def component_blocks(grid: DeviceGrid):
    """[(name, first column, n columns)] of Prophet's predicted components
    (UPSTREAM regressor_column_matrix): each seasonality; each holiday (its
    window columns) and 'holidays' (all of them).  At most PF_MAX_COMP."""
    out, col = [], 0
    for name, _, order in grid.seasons:
        out.append((name, col, 2 * order))
        col += 2 * order
    h = grid.holidays
    if h is not None and h.n:
        h0 = col
        for hn in sorted(set(k.split("_delim_")[0] for k in h.names)):
            idx = [i for i, k in enumerate(h.names) if k.split("_delim_")[0] == hn]
            assert idx == list(range(idx[0], idx[-1] + 1)), "holiday columns not contiguous"
            out.append((hn, h0 + idx[0], len(idx)))
        out.append(("holidays", h0, h.n))
    if len(out) > L.PF_MAX_COMP:
        raise ValueError(f"more than {L.PF_MAX_COMP} components")
    return out


def future_dates(history_dates_ns: np.ndarray, periods: int, freq_ns: int = NS_PER_DAY,
                 include_history: bool = True) -> np.ndarray:
    """UPSTREAM make_future_dataframe: unique history dates + ``periods`` more."""
    h = np.unique(np.asarray(history_dates_ns, np.int64))
    last = int(h[-1])
    fut = last + freq_ns * np.arange(1, periods + 1, dtype=np.int64)
    return np.concatenate((h, fut)) if include_history else fut


# ---------------------------------------------------------------------------
# K2/K3 fit, K4/K5 predict
# ---------------------------------------------------------------------------
@dataclass
class FitResult:
    grid: DeviceGrid
    theta: torch.Tensor      # [n, P] float64
    y_scale: torch.Tensor    # [n]
    f: torch.Tensor          # [n] -log posterior at the returned theta
    f_stan: torch.Tensor     # [n] where the Stan-faithful phase stopped
    status: torch.Tensor     # [n] int32
    n_iter: torch.Tensor
    n_eval: torch.Tensor
    config: ProphetConfig = field(default_factory=ProphetConfig)

    @property
    def P(self):
        return self.theta.shape[1]


class Engine:
    """Batched Prophet engine bound to one GPU."""

    def __init__(self, device: int = 0, config: ProphetConfig | None = None,
                 own_context: bool = False):
        """``own_context``: a private C-ABI context (its own fit workspace), so
        fits of this engine may run concurrently with another engine's on
        other streams (e.g. two ForecastSteps replayed in a pipeline)."""
        self.device = device
        self.owns_context = bool(own_context)
        self.ctx = Context(device) if own_context else Context.get(device)
        self.config = config or ProphetConfig.reference()
        self._vec_cache = {}

    def close(self) -> None:
        """Release a private context (own_context=True); no-op for the shared one."""
        if self.owns_context and not self.ctx.closed:
            torch.cuda.synchronize(self.device)
            self.ctx.close()

    # prior scales and mode indicators (UPSTREAM regressor_column_matrix)
    def _vectors(self, grid: DeviceGrid):
        key = (grid.K, tuple(grid.seasons), self.config.seasonality_mode,
               self.config.seasonality_prior_scale, grid.holidays)
        if key not in self._vec_cache:
            dev = torch.device("cuda", self.device)
            h = grid.holidays
            nh = h.n if h is not None else 0
            ks = grid.K - nh
            mult = self.config.seasonality_mode == "multiplicative"
            sig = [float(self.config.seasonality_prior_scale)] * ks
            m = [1.0 if mult else 0.0] * ks
            if nh:
                hm = h.mode == "multiplicative"
                sig += [float(v) for v in h.prior_scales]
                m += [1.0 if hm else 0.0] * nh
            m = np.asarray(m)
            code = 0 if np.all(m == 1.0) else (1 if np.all(m == 0.0) else 2)
            sig_t = torch.tensor(sig, dtype=torch.float64, device=dev)
            s_m = torch.tensor(m, dtype=torch.float64, device=dev)
            s_a = 1.0 - s_m
            self._vec_cache[key] = (sig_t, s_a, s_m, code)
        return self._vec_cache[key]

    def series_priors(self, grid: DeviceGrid, n: int, changepoint_prior_scale=None,
                      seasonality_prior_scale=None, holidays_prior_scale=None):
        """Per-series prior scales for hyperparameter batching (the AutoML
        ProphetHyperoptEstimator search space, notebooks/automl/...:111-123):
        each argument is a scalar or an [n] array (None: this engine's
        config).  Returns (tau [n], sigmas [n, K]) float64 device tensors for
        ``fit(priors=...)``: Fourier columns get seasonality_prior_scale,
        holiday columns holidays_prior_scale (UPSTREAM's per-holiday default)."""
        dev = torch.device("cuda", self.device)
        cfg = self.config

        def vec(v, default):
            a = np.array(np.broadcast_to(np.asarray(default if v is None else v, np.float64), (n,)))
            if not np.all(a > 0):
                raise ValueError("prior scales must be positive")
            return a
        tau = vec(changepoint_prior_scale, cfg.changepoint_prior_scale)
        sps = vec(seasonality_prior_scale, cfg.seasonality_prior_scale)
        h = grid.holidays
        nh = h.n if h is not None else 0
        sig = np.empty((n, grid.K), np.float64)
        sig[:, :grid.K - nh] = sps[:, None]
        if nh:
            if holidays_prior_scale is None:
                sig[:, grid.K - nh:] = np.asarray(h.prior_scales, np.float64)[None, :]
            else:
                sig[:, grid.K - nh:] = vec(holidays_prior_scale, cfg.holidays_prior_scale)[:, None]
        return _to_device_async(tau, dev), _to_device_async(sig, dev)

    def problem(self, grid: DeviceGrid, y_scaled: torch.Tensor, n: int,
                cap_scaled: torch.Tensor | None = None, priors=None) -> L.PfProblem:
        sig, s_a, s_m, mode = self._vectors(grid)
        pb = L.PfProblem()
        pb.n_series = n
        pb.growth = L.PF_GROWTH[self.config.growth]
        pb.tau = float(self.config.changepoint_prior_scale)
        pb.grid = grid.as_pf()
        pb.sigmas, pb.s_a, pb.s_m = sig.data_ptr(), s_a.data_ptr(), s_m.data_ptr()
        pb.y_scaled = y_scaled.data_ptr()
        if self.config.growth == "logistic":
            if cap_scaled is None:
                raise ValueError("logistic growth needs cap_scaled")
            pb.cap_scaled = cap_scaled.data_ptr()
        else:
            pb.cap_scaled = None
        fo = grid.fourier_orders
        for i in range(3):
            pb.fourier_orders[i] = fo[i]
        pb.season_mode = mode
        pb.tau_series = pb.sigmas_series = None
        if priors is not None:
            tau_s, sig_s = priors
            assert tau_s.dtype == torch.float64 and tuple(tau_s.shape) == (n,)
            assert sig_s.dtype == torch.float64 and tuple(sig_s.shape) == (n, grid.K)
            assert tau_s.is_contiguous() and sig_s.is_contiguous()
            pb.tau_series, pb.sigmas_series = tau_s.data_ptr(), sig_s.data_ptr()
        pb.n_grids = 0
        if isinstance(grid, RaggedGrid):
            pb.n_grids = grid.n_grids
            pb.grids = grid.table.data_ptr()
            pb.grid_of = grid.grid_of.data_ptr()
        pb._keep = (sig, s_a, s_m, y_scaled, cap_scaled, priors, grid)
        return pb

    def prepare(self, grid: DeviceGrid, Y: torch.Tensor, cap: torch.Tensor | None = None):
        """y_scale, y_scaled, Prophet's init theta0, status and (logistic
        growth) cap_scaled on the device.  ``cap`` [n, T_pad] float64 is the
        capacity column (UPSTREAM 'cap'), required for logistic growth."""
        n = Y.shape[0]
        assert Y.dtype == torch.float64 and Y.shape[1] == grid.T_pad and Y.is_contiguous()
        dev = Y.device
        P = 3 + grid.S + grid.K
        y_scale = torch.empty(n, dtype=torch.float64, device=dev)
        y_scaled = torch.empty_like(Y)
        theta = torch.empty((n, P), dtype=torch.float64, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        cap_scaled = None
        if self.config.growth == "logistic":
            if cap is None:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            assert cap.dtype == torch.float64 and cap.shape == Y.shape and cap.is_contiguous()
            cap_scaled = torch.empty_like(Y)
        pg = grid.as_pf()
        ragged = isinstance(grid, RaggedGrid)
        if ragged:
            assert grid.grid_of.numel() == n
        rc = self.ctx.lib.pf_prepare_ragged(
            self.ctx.h, n, ctypes.byref(pg), grid.n_grids if ragged else 0,
            _ptr(grid.table) if ragged else None, _ptr(grid.grid_of) if ragged else None,
            L.PF_GROWTH[self.config.growth], _ptr(Y),
            _ptr(cap) if cap_scaled is not None else None, _ptr(y_scale), _ptr(y_scaled),
            _ptr(cap_scaled) if cap_scaled is not None else None,
            _ptr(theta), _ptr(status), _stream(self.device))
        self.ctx.check(rc, "pf_prepare")
        return y_scale, y_scaled, theta, status, cap_scaled

    def objective_grad(self, grid: DeviceGrid, y_scaled: torch.Tensor, theta: torch.Tensor,
                       cap_scaled: torch.Tensor | None = None, priors=None):
        n = theta.shape[0]
        f = torch.empty(n, dtype=torch.float64, device=theta.device)
        g = torch.empty_like(theta)
        pb = self.problem(grid, y_scaled, n, cap_scaled, priors)
        rc = self.ctx.lib.pf_objective_grad(self.ctx.h, ctypes.byref(pb), _ptr(theta), _ptr(f),
                                            _ptr(g), _stream(self.device))
        self.ctx.check(rc, "pf_objective_grad")
        return f, g

    def hessian(self, grid: DeviceGrid, y_scaled: torch.Tensor, theta: torch.Tensor,
                cap_scaled: torch.Tensor | None = None, priors=None) -> torch.Tensor:
        """[n, P, P] exact Hessian of the smooth part of the -log posterior at
        theta (pf_hessian: the polish's model; Stan's Newton fallback)."""
        n, P = theta.shape
        H = torch.empty((n, P, P), dtype=torch.float64, device=theta.device)
        pb = self.problem(grid, y_scaled, n, cap_scaled, priors)
        rc = self.ctx.lib.pf_hessian(self.ctx.h, ctypes.byref(pb), _ptr(theta), _ptr(H),
                                     _stream(self.device))
        self.ctx.check(rc, "pf_hessian")
        return H

    def fit_opts(self, polish: bool = True, stan_faithful: bool = False, **over) -> L.PfFitOpts:
        """pf_fit_opts: Stan optimizing() defaults + the engine's polish.
        ``stan_faithful`` runs Stan's full L-BFGS termination rules before the
        polish (lbfgs_warmup = 0) instead of the warm-up hand-off."""
        o = L.PfFitOpts()
        self.ctx.lib.pf_default_fit_opts(ctypes.byref(o))
        o.polish = 1 if polish else 0
        if stan_faithful or self.config.growth == "logistic":
            # logistic growth: the warm-up hand-off can certify a worse local
            # optimum than Stan's full run reaches (measured: tests/golden/
            # golden_configs4.npz f_warm60_polish, 1 of 8 series 2.6e-4
            # worse), so the polish starts where Stan's full L-BFGS stops
            o.lbfgs_warmup = 0
        for k, v in over.items():
            setattr(o, k, v)
        return o

    def fit(self, grid: DeviceGrid, Y: torch.Tensor, polish: bool | None = None,
            stan_faithful: bool | None = None, cap: torch.Tensor | None = None, priors=None,
            init=None, **opt) -> FitResult:
        """Fit every row of Y [n, T_pad] (raw y, float64, on this GPU).

        ``polish`` / ``stan_faithful`` default to the config's ``fit_mode``:
        "map" = Stan L-BFGS warm-up (<= lbfgs_warmup iterations) handed to
        the exact-MAP polish (status PF_ST_MAP when certified; uncertified
        series resume L-BFGS); "stan_map" (``stan_faithful=True``) first runs
        Stan's full termination rules (the reference's optimizer run), then
        polishes to the same MAP; "stan" (``polish=False``) stops where Stan
        stops.  ``priors`` (``series_priors``) gives every row its own prior
        scales."""
        mode = self.config.fit_mode
        if polish is None:
            polish = mode != "stan"
        if stan_faithful is None:
            stan_faithful = mode == "stan_map"
        n = Y.shape[0]
        y_scale, y_scaled, theta, status, cap_scaled = self.prepare(grid, Y, cap)
        if init is not None:
            init(theta)
        dev = Y.device
        f = torch.empty(n, dtype=torch.float64, device=dev)
        f_stan = torch.empty(n, dtype=torch.float64, device=dev)
        n_iter = torch.empty(n, dtype=torch.int32, device=dev)
        n_eval = torch.empty(n, dtype=torch.int32, device=dev)
        pb = self.problem(grid, y_scaled, n, cap_scaled, priors)
        o = self.fit_opts(polish, stan_faithful, **opt)
        rc = self.ctx.lib.pf_fit(self.ctx.h, ctypes.byref(pb), ctypes.byref(o), _ptr(theta),
                                 _ptr(f), _ptr(f_stan), _ptr(status), _ptr(n_iter), _ptr(n_eval),
                                 _stream(self.device))
        self.ctx.check(rc, "pf_fit")
        return FitResult(grid, theta, y_scale, f, f_stan, status, n_iter, n_eval, self.config)

    def forecast_async(self, stream: torch.cuda.Stream, fit: FitResult, ds_ns: np.ndarray,
                       **predict_kw):
        """Future grid + ``predict`` on ``stream``, ordered after the work
        queued so far on the current stream (the fit), so the caller's next
        fit overlaps this forecast: the forecast kernels fill the CUs that
        the fit's tail leaves idle (the context's fit scratch is not touched
        by the forecast).  The fit's tensors are recorded on ``stream`` so the
        caching allocator does not hand them out before the forecast has read
        them.  Outputs live on ``stream``: wait on it before using them."""
        cur = torch.cuda.current_stream(fit.theta.device)
        stream.wait_stream(cur)
        g = fit.grid
        gts = g.tensors() if isinstance(g, RaggedGrid) else [g.t, g.XT, g.t_change, g.seg, g.cp_first]
        for t in [fit.theta, fit.y_scale, fit.status] + gts:
            t.record_stream(stream)
        for v in predict_kw.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(stream)
        with torch.cuda.stream(stream):
            fg = self.predict_grid(fit, ds_ns)
            out = self.predict(fit, fg, **predict_kw)
        return fg, out

    def predict_grid(self, fit: FitResult, ds_ns) -> DeviceGrid:
        """Forecast grid on the dates ``ds_ns`` (sorted).  For a ragged fit,
        ``ds_ns`` is a list with the dates of each sub-grid (same order as
        ``fit.grid.grids``); the result is a RaggedGrid of forecast grids."""
        g = fit.grid
        if isinstance(g, RaggedGrid):
            if len(ds_ns) != g.n_grids:
                raise ValueError("ragged predict_grid needs one date array per sub-grid")
            Tp = pad_rows(max(len(d) for d in ds_ns))
            if g.packed is not None:
                p = g.packed
                return RaggedGrid.build(ds_ns, g.seasons, p["starts"], p["scales"], g.grid_of_host,
                                        device=self.device, T_pad=Tp,
                                        changepoint_range=self.config.changepoint_range,
                                        t_change=p["t_change"])
            fgs = [build_grid(d, sg.seasons, start_ns=sg.start_ns, t_scale_ns=sg.t_scale_ns,
                              changepoint_range=self.config.changepoint_range,
                              t_change=sg.t_change, device=self.device, holidays=sg.holidays,
                              T_pad=Tp)
                   for sg, d in zip(g.grids, ds_ns)]
            return RaggedGrid(fgs, g.grid_of_host, self.device)
        return build_grid(ds_ns, g.seasons, start_ns=g.start_ns, t_scale_ns=g.t_scale_ns,
                          changepoint_range=self.config.changepoint_range, t_change=g.t_change,
                          device=self.device, holidays=getattr(g, "holidays", None))

    def predict(self, fit: FitResult, fgrid: DeviceGrid, n_samples: int | None = None,
                seed: int = 0, components: bool = True,
                series_id: torch.Tensor | None = None,
                interval_method: str | None = None,
                cap: torch.Tensor | None = None,
                mc_stream: torch.cuda.Stream | None = None) -> dict:
        """Point forecast + MC intervals for every fitted series on ``fgrid``.
        Returns float32 device tensors [n, fgrid.T_pad] (valid columns :T).
        ``series_id`` (int32/uint32 [n] on the device) keys each series' RNG
        stream so the intervals do not depend on the batch composition.
        ``mc_stream``: launch the Monte-Carlo rows (K5) there, concurrently
        with K4 on the current stream (both only read theta and write disjoint
        rows); the caller joins (``current.wait_stream(mc_stream)``) before
        reading the future rows' intervals."""
        a, out, cap_s = self._predict_args(fit, fgrid, n_samples, seed, components, series_id,
                                           interval_method, cap)
        dev = fit.theta.device
        if mc_stream is None:
            a.parts = 0
            rc = self.ctx.lib.pf_predict(self.ctx.h, ctypes.byref(a), _stream(self.device))
            self.ctx.check(rc, "pf_predict")
            return out
        cur = torch.cuda.current_stream(dev)
        mc_stream.wait_stream(cur)
        a.parts = L.PF_PREDICT_MC
        rc = self.ctx.lib.pf_predict(self.ctx.h, ctypes.byref(a), ctypes.c_void_p(mc_stream.cuda_stream))
        self.ctx.check(rc, "pf_predict (mc part)")
        if not torch.cuda.is_current_stream_capturing():
            # everything K5 reads or writes stays allocated until it ran on the
            # side stream (a captured graph's pool keeps its blocks anyway)
            fgt = fgrid.tensors() if isinstance(fgrid, RaggedGrid) else \
                [fgrid.t, fgrid.XT, fgrid.t_change, fgrid.seg]
            extra = [t for t in (series_id, cap_s) if t is not None]
            for v in list(out.values()) + [fit.theta, fit.y_scale] + fgt + extra:
                v.record_stream(mc_stream)
        a.parts = L.PF_PREDICT_DET
        rc = self.ctx.lib.pf_predict(self.ctx.h, ctypes.byref(a), _stream(self.device))
        self.ctx.check(rc, "pf_predict (det part)")
        return out

    def _predict_args(self, fit: FitResult, fgrid: DeviceGrid, n_samples, seed, components,
                      series_id, interval_method, cap):
        """pf_predict_args for ``predict`` / ``fit_forecast`` and the output
        tensors they name.  Returns (args, out, cap_scaled or None)."""
        n = fit.theta.shape[0]
        dev = fit.theta.device
        if fit.theta.shape[1] != 3 + fgrid.S + fgrid.K:
            # the kernel reads theta with stride 3 + S + K of the forecast grid
            raise ValueError(f"theta has {fit.theta.shape[1]} columns but the forecast grid has "
                             f"3 + S + K = {3 + fgrid.S + fgrid.K} (holiday / extra columns "
                             f"missing from the grid?)")
        ns = self.config.uncertainty_samples if n_samples is None else n_samples
        sig, s_a, s_m, _ = self._vectors(fgrid)
        out = {k: torch.empty((n, fgrid.T_pad), dtype=torch.float32, device=dev)
               for k in ("yhat", "yhat_lower", "yhat_upper")}
        if components:
            for k in ("trend", "trend_lower", "trend_upper", "multiplicative_terms",
                      "additive_terms"):
                out[k] = torch.empty((n, fgrid.T_pad), dtype=torch.float32, device=dev)
        a = L.PfPredictArgs()
        a.n_series = n
        a.growth = L.PF_GROWTH[self.config.growth]
        a.n_samples = int(ns)
        im = self.config.interval_method if interval_method is None else interval_method
        if im not in L.PF_INTERVAL:
            raise ValueError(f"interval_method must be one of {sorted(L.PF_INTERVAL)}")
        a.interval_method = L.PF_INTERVAL[im]
        a.fg = fgrid.as_pf()
        a.s_a, a.s_m = s_a.data_ptr(), s_m.data_ptr()
        a.theta = fit.theta.data_ptr()
        a.y_scale = fit.y_scale.data_ptr()
        cap_s = None
        if self.config.growth == "logistic":
            if cap is None:
                raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
            assert cap.shape == (n, fgrid.T_pad)
            cap_s = (cap.to(torch.float64) / fit.y_scale[:, None]).contiguous()
            a.cap_scaled = cap_s.data_ptr()
        else:
            a.cap_scaled = None
        a.interval_width = float(self.config.interval_width)
        a.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        a.yhat, a.yhat_lower, a.yhat_upper = (out[k].data_ptr() for k in
                                              ("yhat", "yhat_lower", "yhat_upper"))
        if components:
            a.trend, a.trend_lower, a.trend_upper = (out[k].data_ptr() for k in
                                                     ("trend", "trend_lower", "trend_upper"))
            a.mult_terms = out["multiplicative_terms"].data_ptr()
            a.add_terms = out["additive_terms"].data_ptr()
        blocks = component_blocks(fgrid) if components else []
        if blocks:
            comp = torch.empty((len(blocks), n, fgrid.T_pad), dtype=torch.float32, device=dev)
            for b, (name, c0, nc) in enumerate(blocks):
                a.comp_col0[b] = c0
                a.comp_ncol[b] = nc
                out[name] = comp[b]
            a.n_comp = len(blocks)
            a.comp = comp.data_ptr()
        if series_id is not None:
            assert series_id.numel() == n and series_id.dtype == torch.int32 and series_id.is_cuda
            a.series_id = series_id.data_ptr()
        a.n_grids = 0
        if isinstance(fgrid, RaggedGrid):
            if not isinstance(fit.grid, RaggedGrid) or \
                    not np.array_equal(fit.grid.grid_of_host, fgrid.grid_of_host):
                raise ValueError("a ragged forecast grid needs the ragged fit it was built from")
            a.n_grids = fgrid.n_grids
            a.grids = fgrid.table.data_ptr()
            a.grid_of = fgrid.grid_of.data_ptr()
        a._keep = (sig, s_a, s_m, fgrid)
        return a, out, cap_s

    def fit_forecast(self, grid: DeviceGrid, Y: torch.Tensor, fgrid: DeviceGrid, *,
                     n_samples: int | None = None, seed: int = 0, components: bool = True,
                     series_id: torch.Tensor | None = None, interval_method: str | None = None,
                     metrics: bool | str = False, only_fused: bool = False, **opt):
        """``fit`` + ``predict`` on ``fgrid`` (+ with ``metrics`` the in-sample
        metrics of ``diagnostics.insample_metrics`` over the history rows;
        "fast" skips the MDAPE median) through pf_fit_forecast: one launch
        where the layout allows, each series' forecast and metrics computed in
        its fit workgroup as soon as its own fit ends (the same bits as the
        separate launches).  ``fgrid`` must carry the fit grid's changepoints
        (``predict_grid`` / ``build_grid(t_change=grid.t_change)``).
        Returns (FitResult, forecast dict, metrics [n, 7] or None, fused);
        with ``only_fused`` nothing is launched unless fused (then
        (None, None, None, False))."""
        if isinstance(grid, RaggedGrid) or self.config.growth == "logistic":
            if only_fused:
                return None, None, None, False
            fit = self.fit(grid, Y, **opt)
            out = self.predict(fit, fgrid, n_samples=n_samples, seed=seed, components=components,
                               series_id=series_id, interval_method=interval_method)
            met = None
            if metrics:
                from .diagnostics import insample_metrics
                met = insample_metrics(self, Y[:, :grid.T], out["yhat"], out["yhat_lower"],
                                       out["yhat_upper"], mdape=metrics != "fast")
            return fit, out, met, False
        mode = self.config.fit_mode
        polish = opt.pop("polish", None)
        stan_faithful = opt.pop("stan_faithful", None)
        if polish is None:
            polish = mode != "stan"
        if stan_faithful is None:
            stan_faithful = mode == "stan_map"
        n = Y.shape[0]
        y_scale, y_scaled, theta, status, _ = self.prepare(grid, Y)
        dev = Y.device
        f = torch.empty(n, dtype=torch.float64, device=dev)
        f_stan = torch.empty(n, dtype=torch.float64, device=dev)
        n_iter = torch.empty(n, dtype=torch.int32, device=dev)
        n_eval = torch.empty(n, dtype=torch.int32, device=dev)
        fit = FitResult(grid, theta, y_scale, f, f_stan, status, n_iter, n_eval, self.config)
        pb = self.problem(grid, y_scaled, n)
        o = self.fit_opts(polish, stan_faithful, **opt)
        a, out, _ = self._predict_args(fit, fgrid, n_samples, seed, components, series_id,
                                       interval_method, None)
        a.parts = 0
        met, cva = None, None
        if metrics:
            from .diagnostics import insample_args
            met, cva = insample_args(Y[:, :grid.T], out["yhat"], out["yhat_lower"],
                                     out["yhat_upper"], mdape=metrics != "fast")
        fused = ctypes.c_int32(0)
        rc = self.ctx.lib.pf_fit_forecast(
            self.ctx.h, ctypes.byref(pb), ctypes.byref(o), _ptr(theta), _ptr(f), _ptr(f_stan),
            _ptr(status), _ptr(n_iter), _ptr(n_eval), ctypes.byref(a),
            ctypes.byref(cva) if cva is not None else None,
            L.PF_FF_ONLY_FUSED if only_fused else 0, ctypes.byref(fused), _stream(self.device))
        self.ctx.check(rc, "pf_fit_forecast")
        if only_fused and not fused.value:
            return None, None, None, False
        return fit, out, met, bool(fused.value)
