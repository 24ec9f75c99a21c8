"""GPU: the N>1 path end to end with real engine outputs.

Two ranks (one process each, gloo for the collectives, both ranks' engines on
cuda:0 — the box has one GPU; the driver's 8-GPU run uses RCCL) run the
drop-in ``forecast_store_items`` on their splitmix64 hash shard with the
reference's CV metrics, then ``parallel.gather_frames`` / ``gather_blocks``
collect the forecast frames and the metric blocks.  Every rank's gathered
result must equal the world-size-1 run of the whole table bitwise: fits are
per series, and the RNG stream of every series is keyed by its (store, item)
hash, not by its batch position."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_STORES, N_ITEMS = 4, 9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame():
    from distributed_forecasting_amd import synthetic
    return synthetic.store_item_frame(N_STORES, N_ITEMS)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from distributed_forecasting_amd import parallel, training
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fr, met = training.forecast_store_items(_frame(), rank=rank, world_size=world,
                                                cv_metrics=True, return_metrics=True)
        allf = parallel.gather_frames(fr)
        keys = torch.from_numpy(met[["store", "item"]].to_numpy(np.int64))
        vals = torch.from_numpy(met.drop(columns=["store", "item"]).to_numpy(np.float64))
        g = parallel.gather_results(keys, None, metrics=vals)
        q.put((rank, len(fr), {c: allf[c].to_numpy() for c in allf.columns},
               g["keys"].numpy(), g["metrics"].numpy(), g["counts"]))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gather_equals_single_run():
    from distributed_forecasting_amd import batch as B, training
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref, ref_met = training.forecast_store_items(_frame(), cv_metrics=True, return_metrics=True)
    n = N_STORES * N_ITEMS
    keys = ref_met[["store", "item"]].to_numpy(np.int64)
    own = B.shard_of(keys, 2)
    assert 0 < (own == 0).sum() < n
    assert res[0][5] == res[1][5] == [int((own == 0).sum()), int((own == 1).sum())]
    Tf = len(ref) // n
    assert res[0][1] + res[1][1] == len(ref)
    ref_sorted = ref.sort_values(["store", "item", "ds"], kind="stable").reset_index(drop=True)
    ref_m = {tuple(k): ref_met.iloc[i].to_numpy()[2:].astype(np.float64) for i, k in enumerate(keys)}
    for rank, n_local, cols, gk, gm, counts in res:
        import pandas as pd
        got = pd.DataFrame(cols).sort_values(["store", "item", "ds"], kind="stable").reset_index(drop=True)
        assert len(got) == n * Tf
        for c in ("ds", "store", "item"):
            assert np.array_equal(got[c].to_numpy(), ref_sorted[c].to_numpy()), c
        for c in ("y", "yhat", "yhat_upper", "yhat_lower"):
            a, b = got[c].to_numpy(np.float32), ref_sorted[c].to_numpy(np.float32)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) or \
                np.array_equal(a, b, equal_nan=True), c
        assert gk.shape == (n, 2) and gm.shape[0] == n
        for k, m in zip(gk, gm):
            assert np.array_equal(m, ref_m[tuple(int(v) for v in k)], equal_nan=True)


def _nccl_worker(port, q):
    """World size 1 over the nccl backend (RCCL): process group initialised
    before any other GPU call in this process, then the exchange on device
    tensors in every form bench.py / the drop-in use."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        import distributed_forecasting_amd as dfa
        from distributed_forecasting_amd import batch as B, diagnostics, parallel, synthetic
        assert dist.get_backend() == "nccl"
        ds = synthetic.daily_dates("2016-01-01", "2017-12-31")
        n = 24
        Y = synthetic.sales_matrix(n, ds, config_index=1, seed=3)
        keys = np.stack([np.repeat(np.arange(1, 5), 6), np.tile(np.arange(1, 7), 4)], 1)
        sid = torch.from_numpy(B.series_id(keys)).to(dev)
        kd = torch.from_numpy(keys.astype(np.int64)).to(dev)
        eng = dfa.Engine(0)
        with dfa.ForecastStep(eng, ds, n, series_id=sid, metrics="fast") as st:
            st.set_inputs(Y)
            r = st.run()
            o = r["forecast"]
            blk = torch.stack([o["yhat"], o["yhat_lower"], o["yhat_upper"]], 1)
            met = r["metrics"][:, :4].contiguous()
            status = r["fit"].status
            res = {}
            for name, kw in (("all", {}), ("rank0", {"dst": 0}), ("async", {"async_op": True}),
                             ("rank0_async", {"dst": 0, "async_op": True})):
                g = parallel.gather_results(kd, blk, met, status, **kw)
                if kw.get("async_op"):
                    g.wait()
                torch.cuda.synchronize()
                res[name] = all(torch.equal(g[k].view(torch.uint8), v.view(torch.uint8)) for k, v in
                                (("keys", kd), ("forecast", blk), ("metrics", met), ("status", status)))
                res[name + "_bytes"] = g["bytes"]
            # the replayed step + asynchronous gather, as bench.py runs it at N > 1
            st.capture()
            r2 = st.replay()
            o2 = r2["forecast"]
            blk2 = torch.stack([o2["yhat"], o2["yhat_lower"], o2["yhat_upper"]], 1)
            g2 = parallel.gather_results(kd, blk2, r2["metrics"][:, :4].contiguous(), r2["fit"].status,
                                         dst=0, async_op=True).wait()
            torch.cuda.synchronize()
            res["replay"] = torch.equal(g2["forecast"], blk)
        fr = dfa.forecast_store_items(synthetic.store_item_frame(2, 3, "2016-01-01", "2017-12-31"))
        gf = parallel.gather_frames(fr, device=dev)
        res["frames"] = gf.equals(fr)
        q.put(res)
    except Exception as e:  # report in the parent
        import traceback
        q.put({"error": f"{type(e).__name__}: {e}\n{traceback.format_exc()}"})
    finally:
        dist.destroy_process_group()


def test_nccl_world1_gather_on_device():
    """RCCL (backend "nccl") at world size 1 on the box —
    gather_results (all-gather, gather to rank 0, both asynchronous) and
    gather_frames on device tensors equal the non-distributed outputs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    for k in ("all", "rank0", "async", "rank0_async", "replay", "frames"):
        assert res[k] is True, k
    # world size 1: nothing crosses a link
    assert res["all_bytes"] == {"sent": 0, "received": 0}
