"""Multi-GPU sharding: one process per GPU, series
hash-sharded by splitmix64((store << 32) | item) mod world_size, no
cross-GPU traffic until the final gather of forecasts / metrics.

The reference's analogue is Spark's hashpartitioning(store, item) in front of
``applyInPandas`` (notebooks/prophet/02_training.py:305-307); the per-series
validation metrics correspond to what ``train_model`` logs to MLflow
(02_training.py:187-192).  Every exchange is a tensor collective
(``all_gather_into_tensor``: RCCL over xGMI on GPUs, gloo on CPU), padded to
the largest rank's row count; nothing is pickled.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

from . import batch as B


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_indices(keys: np.ndarray, rank: int, world_size: int) -> np.ndarray:
    """Positions of the series this rank owns."""
    return np.flatnonzero(B.shard_of(keys, world_size) == rank)


def gather_counts(n_local: int, device) -> list:
    """Row count of every rank (one tiny all-gather)."""
    ws = dist.get_world_size()
    n = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    cn = torch.zeros(ws, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(cn, n)
    return [int(c) for c in cn.tolist()]


class Gathered(dict):
    """Result of ``gather_results``: keys / forecast / metrics / status (the
    concatenation of every rank's rows in rank order; on ranks other than
    ``dst`` only "counts" and "bytes" when gathering to one rank), "counts",
    and "bytes" = {"sent", "received"} of this rank's share of the exchange.
    With ``async_op=True`` the collectives are in flight: ``wait()`` before
    reading the tensors."""

    def __init__(self):
        super().__init__()
        self._pending = []

    def wait(self) -> "Gathered":
        for work, finish in self._pending:
            if work is not None:
                work.wait()
            finish()
        self._pending = []
        return self


def gather_blocks(local: torch.Tensor, counts=None, dst: int | None = None,
                  async_op: bool = False, _into: Gathered | None = None, _key: str | None = None):
    """Gather a per-rank [n_r, ...] block (padded to max n_r) over the default
    process group (RCCL on GPUs, gloo on CPU): to every rank (``dst=None``,
    all_gather_into_tensor) or to rank ``dst`` only (``dist.gather``).
    Returns (the concatenation of every rank's valid rows in rank order —
    None on ranks other than dst —, per-rank counts, bytes dict)."""
    ws = dist.get_world_size()
    rank = dist.get_rank()
    if counts is None:
        counts = gather_counts(local.shape[0], local.device)
    mx = max(counts)
    rb = int(np.prod(local.shape[1:], dtype=np.int64)) * local.element_size()
    if mx == 0:                       # every rank knows: nothing to exchange
        empty = local.new_empty((0,) + tuple(local.shape[1:]))
        if dst is not None and rank != dst:
            empty = None
        if _into is not None and empty is not None:
            _into[_key] = empty
        return empty, counts, {"sent": 0, "received": 0}
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    if dst is None:
        out = torch.empty((ws * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        work = dist.all_gather_into_tensor(out, pad, async_op=async_op)
        nbytes = {"sent": (ws - 1) * mx * rb, "received": (ws - 1) * mx * rb}
    else:
        out = None
        if rank == dst:
            out = torch.empty((ws * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            work = dist.gather(pad, list(out.chunk(ws, 0)), dst=dst, async_op=async_op)
            nbytes = {"sent": 0, "received": (ws - 1) * mx * rb}
        else:
            work = dist.gather(pad, None, dst=dst, async_op=async_op)
            nbytes = {"sent": mx * rb, "received": 0}

    def finish():
        res = None
        if out is not None:
            res = torch.cat([out[r * mx:r * mx + counts[r]] for r in range(ws)], 0)
        if _into is not None:
            if res is not None:
                _into[_key] = res
        return res
    if async_op:
        if _into is not None:
            _into._pending.append((work, finish))
        return None, counts, nbytes
    return finish(), counts, nbytes


def gather_results(keys: torch.Tensor, forecast: torch.Tensor | None, metrics: torch.Tensor | None = None,
                   status: torch.Tensor | None = None, counts=None, dst: int | None = None,
                   async_op: bool = False) -> Gathered:
    """The engine's final exchange: every rank's
    [S_g, k] int64 series keys, [S_g, 3, T] fp32 forecast blocks (yhat,
    yhat_lower, yhat_upper), [S_g, M] fp64 validation metrics and [S_g]
    int32 fit status.  ``dst=None``: all-gathered to every rank (north_star's
    RCCL all-gather); ``dst=r``: gathered to rank r only (the caller that
    assembles the frame — Spark's driver collecting applyInPandas output):
    rank r receives the same bytes, the other ranks send their block once and
    receive nothing.  One count exchange, then one collective per array.
    ``async_op=True`` leaves the collectives in flight on the backend's stream
    (the caller's next kernels overlap them); ``wait()`` the result first."""
    if counts is None:
        counts = gather_counts(keys.shape[0], keys.device)
    out = Gathered()
    out["counts"] = counts
    tot = {"sent": 0, "received": 0}
    for name, t in (("keys", keys), ("forecast", forecast), ("metrics", metrics), ("status", status)):
        if t is None:
            continue
        res, _, nb = gather_blocks(t, counts, dst=dst, async_op=async_op, _into=out, _key=name)
        if not async_op and res is not None:
            out[name] = res
        tot["sent"] += nb["sent"]
        tot["received"] += nb["received"]
    out["bytes"] = tot
    return out


def gather_frames(frame, key_cols=("store", "item"), device=None):
    """Collect per-rank forecast frames ([ds, *keys, y, yhat, yhat_upper,
    yhat_lower], the applyInPandas schema) on every rank with two tensor
    all-gathers: an int64 block (ds in ns, keys) and a float32 block (the
    value columns).  Returns the concatenated frame in rank order."""
    import pandas as pd
    key_cols = list(key_cols)
    vcols = [c for c in frame.columns if c not in ["ds"] + key_cols]
    dev = torch.device("cpu") if device is None else device
    ints = np.column_stack([frame["ds"].to_numpy("datetime64[ns]").astype(np.int64)] +
                           [frame[k].to_numpy(np.int64) for k in key_cols]) if len(frame) else \
        np.zeros((0, 1 + len(key_cols)), np.int64)
    vals = frame[vcols].to_numpy(np.float32) if len(frame) else np.zeros((0, len(vcols)), np.float32)
    it = torch.from_numpy(np.ascontiguousarray(ints)).to(dev)
    vt = torch.from_numpy(np.ascontiguousarray(vals)).to(dev)
    counts = gather_counts(it.shape[0], dev)
    gi, _, _ = gather_blocks(it, counts)
    gv, _, _ = gather_blocks(vt, counts)
    gi, gv = gi.cpu().numpy(), gv.cpu().numpy()
    out = {"ds": gi[:, 0].astype("datetime64[ns]")}
    for j, k in enumerate(key_cols):
        out[k] = gi[:, 1 + j].astype(frame[k].dtype if len(frame) else np.int32)
    for j, c in enumerate(vcols):
        out[c] = gv[:, j]
    return pd.DataFrame(out)[list(frame.columns)]
