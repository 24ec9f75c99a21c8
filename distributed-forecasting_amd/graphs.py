"""Captured hipGraphs of the fit + forecast step.

A batch of series on one date grid runs ~15 kernels per step (K1 grids,
prepare, the fused fit, forecast grid, K4/K5, K6) whose host side — ctypes
argument structs, torch allocations, Python — costs about as much as the
small launches themselves.  For a serving / training loop that sees batches
of one shape (the reference's nightly refit of every (store, item) on the
same calendar, 02_training.py:305-307), ``ForecastStep`` records the step's
launches once into a hipGraph and replays it: every kernel still runs on
every replay over whatever is in the static input buffer ``Y`` (refresh it
with ``set_inputs``); only the host-side launch work is recorded.

Capture needs the engine's context workspace to be allocated already (no
hipMalloc while capturing): ``capture`` runs the step once eagerly first.
The captured kernels keep pointers into that workspace (the fit's grid
copies), so a step never shares it: when the engine given uses the
per-device shared context, the step runs on a private engine (same config,
its own C-ABI context) — a later, larger fit elsewhere cannot reallocate
the buffers a graph replays on.  A step that made its private engine owns
it: ``close()`` (or garbage collection of the step) drops the graph first and
then destroys that context (pf_ctx_destroy).  RCCL collectives stay outside
the graph (run them after replay).

``fuse`` (default): exact intervals on one grid run fit, forecast and
metrics as ONE launch (pf_fit_forecast, ``fused`` says whether the last step
did): each series' forecast rows and metrics are computed in its fit
workgroup as soon as its own fit ends — the same bits as the separate
launches, which run otherwise (K5 on a side stream, concurrent with K4 / K6).

``metrics``: True (default) computes the whole in-sample set K6 offers
(mse, rmse, mae, mape, smape, coverage and the MDAPE median); "fast" skips
the MDAPE median (NaN) — the set the reference logs (mse / mae / mape,
02_training.py:187-192) plus rmse, smape, coverage; False: no metrics.
"""
from __future__ import annotations

import numpy as np
import torch

from . import engine as E
from . import diagnostics


class ForecastStep:
    """One fit + forecast (+ in-sample metrics) step for a fixed batch shape:
    ``n`` series on the sorted history dates ``ds_ns``, ``horizon`` future
    periods of ``freq_ns``.  ``run()`` launches eagerly; ``replay()`` replays
    the captured graph (``capture()`` first).  Outputs (device tensors, valid
    columns [:Tf]) are in ``out`` after either."""

    def __init__(self, engine: E.Engine, ds_ns: np.ndarray, n: int, *, horizon: int = 90,
                 freq_ns: int = E.NS_PER_DAY, series_id: torch.Tensor | None = None,
                 seed: int = 0, metrics: bool | str = True, interval_method: str | None = None,
                 components: bool = False, fuse: bool = True):
        if metrics not in (True, False, "fast", "all"):
            raise ValueError("metrics must be True, False or 'fast'")
        self._owns_engine = False
        if E.Context._by_device.get(engine.device) is engine.ctx:
            engine = E.Engine(engine.device, engine.config, own_context=True)
            self._owns_engine = True
        self.engine = engine
        cfg = engine.config
        self.ds = np.asarray(ds_ns, np.int64)
        self.T = int(self.ds.shape[0])
        self.seasons = cfg.seasons(int(self.ds[0]), int(self.ds[-1]),
                                   int(np.min(np.diff(self.ds))) if self.T > 1 else 0)
        self.fut = E.future_dates(self.ds, horizon, freq_ns)
        self.Tf = int(self.fut.shape[0])
        dev = torch.device("cuda", engine.device)
        self.Y = torch.zeros((n, E.pad_rows(self.T)), dtype=torch.float64, device=dev)
        self.series_id = series_id
        self.seed = seed
        self.metrics = metrics
        self.interval_method = interval_method
        self.components = components
        self.fuse = fuse
        self.fused = None     # whether the last step ran as one launch (pf_fit_forecast)
        self.graph = None
        self.out = None
        # K5 (Monte-Carlo rows) on a side stream, concurrent with K4 and K6
        self.mc_stream = torch.cuda.Stream(dev)

    def set_inputs(self, Y) -> None:
        """Copy a new batch ([n, T] raw y, host or device) into the static buffer."""
        src = Y if isinstance(Y, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(Y))
        self.Y[:, :self.T].copy_(src, non_blocking=True)

    def _step(self) -> dict:
        eng = self.engine
        grid = E.build_grid(self.ds, self.seasons, start_ns=int(self.ds[0]),
                            t_scale_ns=int(self.ds[-1] - self.ds[0]),
                            n_changepoints=eng.config.n_changepoints,
                            changepoint_range=eng.config.changepoint_range, device=eng.device)
        # the forecast grid needs only the fit grid's changepoints
        cur = torch.cuda.current_stream(self.Y.device)
        fg = E.build_grid(self.fut, self.seasons, start_ns=grid.start_ns,
                          t_scale_ns=grid.t_scale_ns,
                          changepoint_range=eng.config.changepoint_range,
                          t_change=grid.t_change, device=eng.device)
        method = self.interval_method or eng.config.interval_method
        if self.fuse and method == "exact":
            # one launch: each series' forecast rows and metrics run in its fit
            # workgroup as soon as its own fit ends (pf_fit_forecast)
            fit, out, met, fused = eng.fit_forecast(
                grid, self.Y, fg, seed=self.seed, components=self.components,
                series_id=self.series_id, interval_method=self.interval_method,
                metrics=self.metrics, only_fused=True)
            self.fused = fused
            if fused:
                res = {"fit": fit, "forecast": out, "grid": grid, "forecast_grid": fg}
                if self.metrics:
                    res["metrics"] = met
                return res
        self.fused = False
        fit = eng.fit(grid, self.Y)
        out = eng.predict(fit, fg, seed=self.seed, components=self.components,
                          series_id=self.series_id, interval_method=self.interval_method,
                          mc_stream=self.mc_stream)
        res = {"fit": fit, "forecast": out, "grid": grid, "forecast_grid": fg}
        if method == "sample":
            cur.wait_stream(self.mc_stream)     # K5 writes the history rows' intervals too
        if self.metrics:
            # exact intervals: the history rows are written by K4 on this stream
            # the per-series validation metrics the reference logs (mse /
            # mae / mape, 02_training.py:187-192) and rmse, smape, coverage;
            # the MDAPE median unless metrics="fast"
            res["metrics"] = diagnostics.insample_metrics(
                eng, self.Y[:, :self.T], out["yhat"], out["yhat_lower"], out["yhat_upper"],
                mdape=self.metrics != "fast")
        cur.wait_stream(self.mc_stream)
        return res

    def run(self) -> dict:
        """Eager launches (also the warm-up before ``capture``)."""
        self.out = self._step()
        return self.out

    def capture(self) -> "ForecastStep":
        """Record the step into a hipGraph (runs it eagerly once first, on a
        side stream as torch's capture protocol asks)."""
        cur = torch.cuda.current_stream(self.Y.device)
        side = torch.cuda.Stream(self.Y.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self._step()
        cur.wait_stream(side)
        torch.cuda.synchronize(self.Y.device)
        g = torch.cuda.CUDAGraph()
        # thread-local capture: other threads' runtime calls (e.g. the process
        # group's watchdog querying events) do not invalidate the capture
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.out = self._step()
        self.graph = g
        return self

    def replay(self) -> dict:
        if self.graph is None:
            raise RuntimeError("capture() first")
        self.graph.replay()
        return self.out

    def close(self) -> None:
        """Drop the captured graph and the outputs, then destroy the private
        context this step created (a caller-given private engine is left to
        its owner)."""
        if self.graph is not None or self.out is not None:
            torch.cuda.synchronize(self.Y.device)
        self.graph = None
        self.out = None
        if self._owns_engine:
            self.engine.close()

    def __enter__(self) -> "ForecastStep":
        return self

    def __exit__(self, *exc) -> None:
        self.close()
