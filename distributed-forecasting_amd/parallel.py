"""Multi-GPU sharding: one process per GPU, series
hash-sharded by splitmix64((store << 32) | item) mod world_size, no
cross-GPU traffic until the final gather of forecasts / metrics.

The reference's analogue is Spark's hashpartitioning(store, item) in front of
``applyInPandas`` (notebooks/prophet/02_training.py:305-307).
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


def gather_blocks(local: torch.Tensor, counts=None):
    """All-gather a per-rank [n_r, ...] block (padded to max n_r) over the
    default process group (RCCL on GPUs, gloo on CPU).  Returns (the
    concatenation of every rank's valid rows, per-rank counts)."""
    ws = dist.get_world_size()
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    if counts is None:
        cn = [torch.zeros_like(n) for _ in range(ws)]
        dist.all_gather(cn, n)
        counts = [int(c.item()) for c in cn]
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((ws * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad)
    parts = [out[r * mx:r * mx + counts[r]] for r in range(ws)]
    return torch.cat(parts, 0), counts


def gather_frames(frame):
    """Collect per-rank pandas frames on every rank (result assembly for the
    pandas-level API; the bulk data path uses gather_blocks)."""
    import pandas as pd
    ws = dist.get_world_size()
    objs = [None] * ws
    dist.all_gather_object(objs, frame)
    return pd.concat(objs, ignore_index=True)
