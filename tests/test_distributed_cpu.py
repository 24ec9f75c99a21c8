"""CPU: the N>1 path (hash sharding + final gather) with world_size-2 gloo."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_forecasting_amd import batch as B, parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = np.stack(np.meshgrid(np.arange(1, 11), np.arange(1, 51), indexing="ij"),
                        -1).reshape(-1, 2)
        mine = parallel.shard_indices(keys, rank, world)
        # stand-in for the per-rank forecast block: [n_r, 3] = (store, item, f(store, item))
        k = keys[mine]
        local = torch.from_numpy(np.column_stack([k, k[:, 0] * 1000 + k[:, 1]]).astype(np.float32))
        allb, counts = parallel.gather_blocks(local)
        q.put((rank, mine.tolist(), allb.numpy().tolist(), counts))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    m0, m1 = set(res[0][1]), set(res[1][1])
    assert not (m0 & m1) and len(m0 | m1) == 500
    assert res[0][3] == res[1][3] == [len(m0), len(m1)]
    for r in res:
        rows = np.array(r[2])
        assert rows.shape == (500, 3)
        assert np.array_equal(rows[:, 2], rows[:, 0] * 1000 + rows[:, 1])
        assert len({(a, b) for a, b in rows[:, :2].astype(int)}) == 500
