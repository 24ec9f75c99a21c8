"""Benchmark: series fit+forecast per second on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One step = the whole hot path for this rank's batch of series, inputs resident
in HBM: K1 design grid (history) -> prepare/init -> K3 fit (Stan L-BFGS warm-up
handed to the certified exact-MAP polish) -> K1 future grid -> K4/K5 90-day
forecast with 1000-sample 95% intervals -> K6 per-series validation metrics
(in-sample mse/rmse/mae/mape) -> (N>1) RCCL all-gather of the keys, forecast
blocks, metrics and status.

Headline workload: BASELINE.json configs[1] — 500 synthetic Kaggle-shaped
series x 1826 days per GPU (SURVEY.md §8d generator); N>1: weak scaling, 500
series per GPU (10*N stores x 50 items) hash-sharded by (store, item).

Also timed in the same run and reported beside ``value`` (same bracketing:
barrier + synchronize, max over ranks):
  full_sampling   every row's 1000 samples materialised
  stan_full       Stan's full L-BFGS termination rules before the polish
  dropin          the reference's own surfaces on the same series: the
                  batched applyInPandas equivalent forecast_store_items(df)
                  (pandas in, DataFrame out; N>1: this rank's hash shard +
                  tensor all-gather of the frames), the PyFunc
                  ForecastStoreItemModel.predict from a params store
                  (model_wrapper.py:43-73), and the CV-on training step
                  (fit + 3 CV refits/forecasts + K6 metrics + forecast,
                  02_training.py:172-205)
  configs2_strong BASELINE configs[2]: 50,000 series x 1826 days in total,
                  hash-sharded over the N ranks (strong scaling), per-rank
                  counts reported
roofline: the dominant kernel (k_fit_forecast: fit + polish + each series' forecast
rows and metrics in one launch; k_fit_polish when unfused), timed with HIP events recorded by
the engine on the launch stream.  achieved = SURVEY §8d algorithmic FLOPs (the
oracle Stan run's evaluation count E per series x 4T(F+2C)) / kernel time;
achieved_performed = the evaluations the engine actually ran.
cpu_baseline: the CPU restatement (oracle/: Stan L-BFGS in C + numpy 1000-sample
predictive sampler), timed in a process pool on all 500 series, rank 0, N=1;
the same run feeds the accuracy distributions (MAP vs Stan endpoint).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T_DAYS = 1826
HORIZON = 90
N_SAMPLES = 1000
SERIES_PER_GPU = 500
C2_SERIES = 50_000
FLOPS_PER_EVAL = 4 * T_DAYS * (26 + 2 * 25)      # 555,104
PEAK_VALU_GINSTS = 1024 * 2.4 / 2    # wave64 VALU instructions per ns, whole GPU
PEAK_FP64_TFLOPS = 78.6                            # MI355X FP64 (vector = matrix), SURVEY.md §8d
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--series-per-gpu", type=int, default=SERIES_PER_GPU)
    ap.add_argument("--cpu-sample", type=int, default=500,
                    help="series in the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="0: every CPU this process may use (cpu_share())")
    ap.add_argument("--cpu-cv-sample", type=int, default=128,
                    help="series in the CV-on CPU-baseline sample (0 disables)")
    ap.add_argument("--gather", choices=("rank0", "all"), default="rank0",
                    help="N>1 exchange: gather to rank 0 (the frame's consumer) or all-gather")
    ap.add_argument("--dropin-steps", type=int, default=10)
    ap.add_argument("--c2-steps", type=int, default=3)
    ap.add_argument("--c2-series", type=int, default=C2_SERIES)
    ap.add_argument("--no-variants", action="store_true",
                    help="headline only (profiling runs)")
    return ap.parse_args()


# --------------------------------------------------------------- workload
def keys_for(n_total: int):
    n_items = 50
    n_stores = max(1, (n_total + n_items - 1) // n_items)
    return np.stack(np.meshgrid(np.arange(1, n_stores + 1), np.arange(1, n_items + 1),
                                indexing="ij"), -1).reshape(-1, 2)[:n_total]


def workload(world: int, per_gpu: int, config_index: int = 1):
    from distributed_forecasting_amd import synthetic
    keys = keys_for(per_gpu * world)
    ds = synthetic.daily_dates()
    Y = synthetic.sales_matrix(len(keys), ds, config_index=config_index)
    return keys, ds, Y


# ------------------------------------------------------------ CPU baseline
def _cpu_one(args):
    """One series through the CPU restatement: Stan L-BFGS fit (C) +
    make_future_dataframe(90) + 1000-sample predictive intervals (numpy)."""
    ds, y, seed = args
    from oracle import prophet_oracle as po, stan_oracle as so
    st = po.build_problem(ds, y)
    th = so.fit_setup(st)[0]
    par = po.params_from_theta(th, st.problem.S)
    fut = po.make_future_dates(ds, HORIZON)
    out = po.sample_uncertainty(st, par, fut, n_samples=N_SAMPLES,
                                rng=np.random.default_rng(seed))
    return out["yhat"], th


def _cpu_extra(args):
    """Untimed: the oracle's certified MAP (polish from its Stan endpoint)
    and Stan restarted from an init perturbed by 1e-14 (Stan's own rounding
    sensitivity); point forecasts of both."""
    ds, y, th_stan = args
    from oracle import prophet_oracle as po, stan_oracle as so
    st = po.build_problem(ds, y)
    thm = so.polish(st.problem, th_stan, 50, damp=True)[0]
    th0 = st.theta0.copy()
    th0[0] *= 1.0 + 1e-14
    thp = so.lbfgs(st.problem, th0)[0]
    fut = po.make_future_dates(ds, HORIZON)
    yh = [po.predict_point(st, po.params_from_theta(t, st.problem.S), fut)["yhat"] for t in (thm, thp)]
    return yh[0], yh[1], st.hist.y_scale


def _cpu_one_cv(args):
    """One series with the reference's train_model CV (02_training.py:178-188):
    3 fold refits (UPSTREAM cross_validation: horizon 90 d, period 360 d,
    initial 730 d), each fold's 90-row forecast with 1000-sample intervals,
    performance_metrics + the notebook's mean over horizons; then the full
    fit + 90-day forecast with intervals (as _cpu_one)."""
    ds, y, seed = args
    from oracle import prophet_oracle as po, stan_oracle as so
    rng = np.random.default_rng(seed)
    H = HORIZON * po.NS_PER_DAY
    cut = po.generate_cutoffs(ds, H, 730 * po.NS_PER_DAY, 360 * po.NS_PER_DAY)
    ys, fs, hs = [], [], []
    for c in cut:
        tr = ds <= c
        te = (ds > c) & (ds <= c + H)
        st = po.build_problem(ds[tr], y[tr])
        th = so.fit_setup(st)[0]
        o = po.sample_uncertainty(st, po.params_from_theta(th, st.problem.S), ds[te],
                                  n_samples=N_SAMPLES, rng=rng)
        ys.append(y[te]); fs.append(o["yhat"]); hs.append(ds[te] - c)
    pm = po.performance_metrics(np.concatenate(ys), np.concatenate(fs), np.concatenate(hs),
                                metrics=("mse", "mae", "mape"))
    met = {m: float(np.mean(pm[m])) for m in ("mse", "mae", "mape") if m in pm}
    yh, th = _cpu_one((ds, y, seed + 1))
    return met, yh


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota and by OMP_NUM_THREADS when the environment sets them (on the GPU
    box os.cpu_count() reports the whole machine, not this job's share)."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_quota"] = quota
    omp = os.environ.get("OMP_NUM_THREADS")
    info["omp_num_threads"] = int(omp) if omp and omp.isdigit() else None
    n = info["affinity"]
    if quota:
        n = min(n, max(1, int(quota)))
    if info["omp_num_threads"]:
        n = min(n, info["omp_num_threads"])
    info["usable"] = n
    return info


def cpu_baseline_cv(ds, Y, n_sample: int, workers: int):
    import multiprocessing as mp
    jobs = [(ds, Y[i], 5000 + 7 * i) for i in range(n_sample)]
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        pool.map(_cpu_one, [(ds, Y[i], 1) for i in range(workers)])
        t0 = time.perf_counter()
        res = pool.map(_cpu_one_cv, jobs, chunksize=1)
        dt = time.perf_counter() - t0
    return dict(rate=n_sample / dt, dt=dt, n=n_sample,
                metric_means={k: float(np.nanmean([r[0][k] for r in res])) for k in res[0][0]})


def cpu_baseline(ds, Y, n_sample: int, workers: int):
    import multiprocessing as mp
    from oracle import stan_oracle as so
    so.lib()                                   # build/load the C oracle once
    jobs = [(ds, Y[i], 1000 + i) for i in range(n_sample)]
    ctx = mp.get_context("fork")               # no exec; runs before any GPU init
    with ctx.Pool(workers) as pool:
        pool.map(_cpu_one, jobs[:workers])     # warm the workers (imports)
        t0 = time.perf_counter()
        res = pool.map(_cpu_one, jobs, chunksize=1)
        dt = time.perf_counter() - t0
        extra = pool.map(_cpu_extra, [(ds, Y[i], res[i][1]) for i in range(n_sample)], chunksize=4)
    return dict(rate=n_sample / dt, dt=dt, yhat_stan=np.stack([r[0] for r in res]),
                yhat_map=np.stack([e[0] for e in extra]), yhat_pert=np.stack([e[1] for e in extra]),
                y_scale=np.array([e[2] for e in extra]))


def dist_stats(d):
    d = np.asarray(d)
    return {"max": float(d.max()), "p50": float(np.median(d)), "p90": float(np.quantile(d, 0.9)),
            "frac_gt_1e-3": float((d > 1e-3).mean()), "n_series": int(d.size)}


# ------------------------------------------------------------------ main
def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)

    keys, ds, Y_all = workload(world, args.series_per_gpu)

    # CPU baseline first (rank 0, N=1): forked workers, before the GPU is touched
    cpu = None
    if world == 1 and rank == 0 and args.cpu_sample > 0:
        share = cpu_share()
        workers = args.cpu_workers or share["usable"]
        n_s = min(max(args.cpu_sample, workers), len(keys))
        cpu = cpu_baseline(ds, Y_all, n_s, workers)
        cpu["n"] = n_s
        cpu["workers"] = workers
        cpu["share"] = share
        if args.cpu_cv_sample > 0:
            cpu["cv"] = cpu_baseline_cv(ds, Y_all, min(args.cpu_cv_sample, len(keys)), workers)

    import torch
    import torch.distributed as dist
    import distributed_forecasting_amd as dfa
    from distributed_forecasting_amd import batch as B, diagnostics, parallel

    dev = local
    torch.cuda.set_device(dev)
    device = torch.device("cuda", dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    mine = parallel.shard_indices(keys, rank, world) if world > 1 else np.arange(len(keys))
    n = len(mine)
    eng = dfa.Engine(dev)                       # reference config (02_training.py:162-169)
    cfg = eng.config
    seasons = cfg.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    T = len(ds)
    Tp = dfa.pad_rows(T)

    def resident(Y):
        Yd = torch.zeros((Y.shape[0], Tp), dtype=torch.float64, device=device)
        Yd[:, :T] = torch.from_numpy(Y).to(device)
        return Yd

    Yd = resident(Y_all[mine])
    sid = torch.from_numpy(B.series_id(keys[mine])).to(device)
    kd = torch.from_numpy(keys[mine].astype(np.int64)).to(device)
    fut = B.future_dates(ds, HORIZON)
    torch.cuda.synchronize()

    def step(Yd=Yd, sid=sid, kd=kd, method="exact", stan_faithful=None, counts=None):
        grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]),
                              device=dev)
        fit = eng.fit(grid, Yd, stan_faithful=stan_faithful)
        fg = eng.predict_grid(fit, fut)
        out = eng.predict(fit, fg, seed=0, components=False, series_id=sid,
                          interval_method=method)
        met = diagnostics.insample_metrics(eng, Yd[:, :T], out["yhat"], out["yhat_lower"],
                                           out["yhat_upper"], mdape=False)
        if world > 1:
            blk = torch.stack([out["yhat"], out["yhat_lower"], out["yhat_upper"]], 1)
            parallel.gather_results(kd, blk, met[:, :4].contiguous(), fit.status, counts=counts, dst=dst)
        return fit, fg, out, met

    def bracket():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.int64, device=device)
        dist.all_reduce(t)
        return int(t.item())

    counts = parallel.gather_counts(n, device) if world > 1 else None

    # per-kernel averages over the timed steps (HIP events on the launch stream)
    def averages(records):
        kern = {}
        for name, ms, grid_n in records:
            k = kern.setdefault(name, [0.0, 0])
            k[0] += ms
            k[1] += 1
        return {k: v[0] / v[1] for k, v in kern.items()}

    def timed(fn, steps, warm=1, ctx=None, drain=None, kernels=True):
        """Same bracketing as the headline: warm-up, barrier + sync, `steps`
        calls, barrier + sync, max over ranks; kernel averages from the HIP
        events of the engine context the launches go through (``kernels``:
        off for the host-bound drop-in legs, whose launches would each pay
        two event records).  ``drain`` completes work still in flight
        (asynchronous exchanges) inside the timed region."""
        ctx = ctx or eng.ctx
        for _ in range(warm):
            fn()
        if drain:
            drain()
        bracket()
        ctx.set_timing(kernels)
        t0_ = time.perf_counter()
        r = None
        for _ in range(steps):
            r = fn()
        if drain:
            drain()
        bracket()
        el = time.perf_counter() - t0_
        ka = averages(ctx.read_timings())
        ctx.set_timing(False)
        return max_over_ranks(el), ka, r

    # ---------------------------------------------------------- headline
    # the same step as a captured hipGraph (graphs.ForecastStep: every kernel
    # runs on every replay; the host-side launch work is recorded once), the
    # RCCL gather after the replay; the eager launches are timed first (their
    # HIP events give the per-kernel times the roofline uses)
    fstep = dfa.ForecastStep(eng, ds, n, horizon=HORIZON, series_id=sid, metrics="fast")
    fstep.set_inputs(Yd[:, :T])

    def unpack(r):
        return r["fit"], r["forecast_grid"], r["forecast"], r["metrics"]

    dst = 0 if args.gather == "rank0" else None
    pending = []
    xbytes = {}

    def gather(r):
        # the exchange runs asynchronously on RCCL's stream: the copies below
        # snapshot this step's outputs (the replayed graph rewrites its static
        # buffers), so step k's gather overlaps step k+1's kernels
        if world > 1:
            o = r["forecast"]
            blk = torch.stack([o["yhat"], o["yhat_lower"], o["yhat_upper"]], 1)
            g = parallel.gather_results(kd, blk, r["metrics"][:, :4].contiguous(),
                                        r["fit"].status.clone(), counts=counts, dst=dst,
                                        async_op=True)
            pending.append(g)
            xbytes.update(g["bytes"])
        return r

    def drain():
        while pending:
            pending.pop(0).wait()

    def stepped(fn):
        def run():
            r = fn()
            if len(pending) > 2:            # bound the in-flight exchanges
                pending.pop(0).wait()
            return r
        return run

    sctx = fstep.engine.ctx                 # the step's private context (graphs.py)
    el_eager, kern_avg, _ = timed(stepped(lambda: gather(fstep.run())), args.steps, args.warmup,
                                  sctx, drain=drain)
    launch = "hipGraph replay"
    try:
        fstep.capture()
        elapsed, _, r = timed(stepped(lambda: gather(fstep.replay())), args.steps, args.warmup,
                              sctx, drain=drain)
    except Exception as e:                  # capture unsupported: report the eager step
        launch = f"eager (graph capture failed: {type(e).__name__}: {e})"
        elapsed, r = el_eager, fstep.run()
    fit, fg, out, met = unpack(r)
    total_series = sum_over_ranks(n)
    value = total_series * args.steps / elapsed
    # the same step as separate launches (fit | K4 + K6 || K5 on a side
    # stream): the per-kernel times of the forecast kernels, and the gain of
    # the fused launch
    ustep = dfa.ForecastStep(eng, ds, n, horizon=HORIZON, series_id=sid, metrics="fast", fuse=False)
    ustep.set_inputs(Yd[:, :T])
    el_unf, kern_unf, _ = timed(stepped(lambda: gather(ustep.run())), args.steps, args.warmup,
                                ustep.engine.ctx, drain=drain)
    try:
        ustep.capture()
        el_unf_g, _, _ = timed(stepped(lambda: gather(ustep.replay())), args.steps, args.warmup,
                               ustep.engine.ctx, drain=drain)
    except Exception:                       # capture unsupported: the eager figure
        el_unf_g = el_unf
    ustep.close()

    res = {
        "metric": "series fit+forecast/sec (1826d daily, 90d horizon, 1000-sample 95% intervals)",
        "value": value, "unit": "series/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md §8d Kaggle-shaped generator, seed 20261015+1)",
        "config": {"workload": "configs[1]: 500 series x 1826 days per GPU, Prophet MAP fit "
                               "(Stan L-BFGS warm-up + certified exact-MAP polish) + 90-day "
                               "forecast with 1000-sample 95% intervals + per-series validation "
                               "metrics (reference Prophet config, 02_training.py:162-169)",
                   "intervals": "exact: history rows (deterministic trend) draw the order "
                                "statistics of the 1000 noise samples exactly (same law); the "
                                "90 future rows materialise all 1000 samples",
                   "series_per_gpu": args.series_per_gpu, "series_total": total_series,
                   "series_this_rank": n, "series_per_rank": counts or [n], "T": T,
                   "horizon": HORIZON, "uncertainty_samples": N_SAMPLES,
                   "parallelism": f"dp{world} (series hash-sharded by (store, item); RCCL "
                                  f"all-gather of keys, forecasts, metrics, status)"},
        "kernels_ms": kern_avg,
        "metrics": {"kind": "in-sample",
                    "set": ["mse", "rmse", "mae", "mape"],
                    "note": "per-series validation metrics computed in the timed step (K6 over the "
                            "history rows: mse, rmse, mae, mape, smape, coverage; the MDAPE median "
                            "is not computed — the reference logs mse / mae / mape) and, at N>1, "
                            "RCCL-all-gathered with the keys; the "
                            "reference's cross-validation metrics (02_training.py:178-188: 3 fold "
                            "refits) are the dropin.forecast_store_items_cv and cv_on legs"},
        "launch": launch,
        "fused": bool(fstep.fused),
        "unfused": {"value": total_series * args.steps / el_unf_g, "unit": "series/s",
                    "ms_per_step": el_unf_g / args.steps * 1e3, "kernels_ms": kern_unf,
                    "note": "the same step as separate launches (k_fit_polish, then k_predict_det "
                            "+ k_cv_metrics on the step's stream and k_predict_mc on a side "
                            "stream), graph-replayed; the headline runs them as one launch "
                            "(pf_fit_forecast, k_fit_forecast: bitwise the same outputs)"},
        "eager": {"value": total_series * args.steps / el_eager, "unit": "series/s",
                  "ms_per_step": el_eager / args.steps * 1e3,
                  "note": "the same step launched eagerly (Python + ctypes per launch); "
                          "kernels_ms and the roofline come from these launches' HIP events"},
    }

    # ------------------------------------------------------ exchange bytes
    # per series: int64 keys (16 B), the [3, T_pad] fp32 forecast block,
    # 4 fp64 metrics, int32 status; projected for the 8-GPU weak-scaling run
    # (500 series per GPU, splitmix64 shards padded to the largest rank)
    row_b = 16 + 3 * int(out["yhat"].shape[1]) * 4 + 4 * 8 + 4
    k8 = keys_for(8 * args.series_per_gpu)
    mx8 = int(np.bincount(B.shard_of(k8, 8), minlength=8).max())
    proj8 = 7 * mx8 * row_b
    link_gbs = 64.0        # assumed sustained one-direction xGMI rate per peer link (GB/s)
    res["exchange"] = {
        "mode": ("gather to rank 0" if dst == 0 else "all-gather") +
                " (RCCL, asynchronous: overlaps the next step's kernels)",
        "bytes_per_step_this_rank": xbytes if world > 1 else {"sent": 0, "received": 0},
        "bytes_per_series": row_b,
        "projected_n8": {"max_rank_series": mx8, "rank0_received_bytes_per_step": proj8,
                         "other_rank_sent_bytes_per_step": mx8 * row_b,
                         "projected_ms_at_7_links": proj8 / (7 * link_gbs * 1e9) * 1e3,
                         "assumed_link_GBps": link_gbs,
                         "note": "all-gather: every rank receives the rank-0 figure"}}

    # ---------------------------------------------------------- roofline
    with open(os.path.join(ROOT, "tests", "golden", "bench_manifest.json")) as f:
        man = json.load(f)
    E_all = np.array(man["E"], dtype=np.float64)
    E_mean = float(E_all.mean())
    evals = float(fit.n_eval.double().sum().item())
    fit_kernel = next(k for k in ("k_fit_forecast", "k_fit_polish", "k_fit") if k in kern_avg)
    fit_s = kern_avg.get(fit_kernel, float("nan")) / 1e3
    # algorithmic work per series = E x 4T(F+2C), E = the
    # oracle's Stan-faithful evaluation count for that series (fixed per
    # series, tests/golden/bench_manifest.json) -- the Stan fit the launch
    # replaces; the engine performs fewer evaluations (warm-up + polish)
    mine_E = E_all[mine] if len(E_all) >= len(keys) else np.full(n, E_mean)
    flops_alg = float(mine_E.sum()) * FLOPS_PER_EVAL
    flops = evals * FLOPS_PER_EVAL
    achieved = flops_alg / fit_s / 1e12
    achieved_perf = flops / fit_s / 1e12
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_k_fit.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    res["roofline"] = {
        "bound": "mfma",
        "kernel_ms_source": "HIP events of the eager headline launches (same kernels as the "
                            "graph replay; profiles/ rocprofv3 trace of the replayed run)", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
        "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic, "kernel": fit_kernel,
        "kernel_ms": kern_avg.get(fit_kernel), "flops_per_launch": flops_alg,
        "evals_algorithmic_per_launch": float(mine_E.sum()),
        "evals_performed_per_launch": evals,
        "achieved_performed": achieved_perf, "frac_performed": achieved_perf / PEAK_FP64_TFLOPS,
        "limiter": "latency: per evaluation a 4-wave row pass then a serial wave-0 L-BFGS step "
                   "(profiles/ SQ counters: wait-dominated); the row pass's contractions are "
                   "FP64 VALU, FP64 MFMA only in the polish Hessian",
        "note": "bound 'mfma' = compute-bound against the FP64 peak (MI355X FP64 vector peak = "
                "FP64 matrix peak = 78.6 TF).  frac = SURVEY §8d algorithmic FLOPs (the oracle "
                "Stan run's evaluations E per series x 4T(F+2C)) / the fused fit+polish kernel's "
                "time; frac_performed = the kernel-efficiency figure on the L-BFGS evaluations "
                "the engine performed; traffic = HBM bytes per launch from rocprofv3 PMC "
                "(profiles/pmc_k_fit.json).  k_fit_forecast also runs each series' forecast "
                "rows and metrics (K4/K5/K6) after its fit: its time includes them, its FLOPs "
                "count only the fit's (conservative)"}
    # K5 (the Monte-Carlo future rows, the longest forecast kernel) is
    # VALU-issue-bound work (Philox, Box-Muller, wave sorts): its roofline is
    # the vector-instruction issue rate, one wave64 VALU instruction per 2
    # cycles per SIMD (1024 SIMDs at 2.4 GHz), with the instruction count per
    # launch from rocprofv3 PMC (SQ_INSTS_VALU, profiles/pmc_k_predict_mc.json,
    # same launch shape) over the live kernel time
    mc_ms = kern_unf.get("k_predict_mc")
    mc_pmc = None
    mc_path = os.path.join(ROOT, "profiles", "pmc_k_predict_mc.json")
    if os.path.exists(mc_path):
        with open(mc_path) as f:
            mc_pmc = json.load(f)
    if mc_ms and mc_pmc and mc_pmc.get("n_series") == n and mc_pmc.get("horizon") == HORIZON:
        insts = float(mc_pmc["SQ_INSTS_VALU"])
        ach = insts / (mc_ms / 1e3)
        res["forecast_roofline"] = {
            "bound": "valu-issue", "kernel": "k_predict_mc", "kernel_ms": mc_ms,
            "achieved": ach / 1e9, "peak": PEAK_VALU_GINSTS, "unit": "G wave-instr/s",
            "frac": ach / 1e9 / PEAK_VALU_GINSTS, "valu_insts_per_launch": insts,
            "pmc": f"profiles/pmc_k_predict_mc.json ({mc_pmc.get('tag')})",
            "note": "VALU issue rate = SQ_INSTS_VALU per launch (rocprofv3 PMC) / the kernel's "
                    "live HIP-event time, against 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 "
                    "instruction; K4 (k_predict_det) and K6 run concurrently on the other stream"}
    else:
        res["forecast_roofline"] = None
    res["fit_stats"] = {"n_eval_mean": float(fit.n_eval.float().mean().item()),
                        "n_eval_max": int(fit.n_eval.max().item()),
                        "map_certified": float((fit.status == 70).float().mean().item()),
                        "E_oracle_stan_full_mean": E_mean}
    headline_yhat = out["yhat"][:, :fg.T].double().cpu().numpy()

    if not args.no_variants:
        # every row's intervals materialised from N samples (UPSTREAM's
        # literal loop), and the reference-shaped optimizer run (Stan's full
        # L-BFGS termination rules before the polish)
        el, ka, _ = timed(lambda: step(method="sample", counts=counts), args.steps)
        res["full_sampling"] = {"value": total_series * args.steps / el, "unit": "series/s",
                                "ms_per_step": el / args.steps * 1e3, "kernels_ms": ka,
                                "note": "interval_method='sample': all 1916 rows x 1000 samples "
                                        "materialised per series (UPSTREAM's literal loop)"}
        el, ka, _ = timed(lambda: step(stan_faithful=True, counts=counts), args.steps)
        res["stan_full"] = {"value": total_series * args.steps / el, "unit": "series/s",
                            "ms_per_step": el / args.steps * 1e3, "kernels_ms": ka,
                            "note": "fit_mode='stan_map': Stan's full L-BFGS termination rules "
                                    "(the reference's optimizer run, ~350 evals/series) before "
                                    "the polish; same MAP as the headline"}
        res["dropin"] = dropin(args, eng, keys[mine], ds, Y_all[mine], Yd, rank, world, bracket,
                               max_over_ranks, sum_over_ranks, timed, parallel, device)
        res["configs2_strong"] = configs2(args, eng, ds, seasons, fut, rank, world, device, timed,
                                          sum_over_ranks, parallel, B, diagnostics, dfa)
        res["ragged"] = ragged_leg(args, eng, device, timed, sum_over_ranks, B, dfa)

    if cpu is not None:
        m = cpu["n"]
        ysc = cpu["y_scale"]
        st_mode = stan_mode_yhat(dfa, eng.config, ds, seasons, Yd[:m], fut, dev)
        rel = lambda a, b: np.abs(a - b).max(1) / ysc  # noqa: E731
        res["accuracy"] = {
            "map_vs_oracle_stan_endpoint": dist_stats(rel(headline_yhat[:m], cpu["yhat_stan"])),
            "map_vs_oracle_map": dist_stats(rel(headline_yhat[:m], cpu["yhat_map"])),
            "stan_mode_vs_oracle_stan_endpoint": dist_stats(rel(st_mode, cpu["yhat_stan"])),
            "oracle_stan_vs_itself_init_perturbed_1e-14": dist_stats(rel(cpu["yhat_pert"],
                                                                        cpu["yhat_stan"])),
            "note": "rel = max_t |yhat_a - yhat_b| / y_scale per series, over all bench series. "
                    "The headline returns the certified MAP; fit_mode='stan' stops where Stan's "
                    "L-BFGS stops (the reference-shaped answer).  Stan's endpoint itself moves "
                    "by the last line's amount when its init is perturbed by 1e-14 (its "
                    "termination at the |delta| kink is rounding-sensitive)."}
        cv = cpu.get("cv")
        res["cpu_baseline"] = {
            "value": cpu["rate"], "unit": "series/s", "cores": cpu["workers"], "kind": "port",
            "sample": (f"all {m} bench series; per series: Stan L-BFGS MAP (oracle C "
                       f"restatement) + 90-day forecast with {N_SAMPLES}-sample intervals (numpy "
                       f"restatement); {cpu['workers']}-process pool (Spark local[{cpu['workers']}] "
                       f"shape: one series per task), {cpu['dt']:.1f} s wall; CV off"),
            "cpu_share": cpu["share"],
            "cv_on": None if cv is None else {
                "value": cv["rate"], "unit": "series/s", "cores": cpu["workers"], "n_series": cv["n"],
                "wall_s": cv["dt"], "cv_metric_means": cv["metric_means"],
                "sample": (f"first {cv['n']} bench series; per series the reference's train_model: "
                           f"3 CV fold refits (1016/1376/1736 rows) each with a 90-row "
                           f"{N_SAMPLES}-sample forecast + performance_metrics (mse/mae/mape), then "
                           f"the full fit + 90-day forecast with intervals (02_training.py:172-205)")},
            "note": ("cores = the CPUs this process may use (affinity, capped by the cgroup quota "
                     "and OMP_NUM_THREADS: the box's share; os_cpu_count is the whole machine)")}
    else:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


def stan_mode_yhat(dfa, cfg0, ds, seasons, Yd, fut, dev):
    """Untimed: fit_mode='stan' (Stan's L-BFGS only) point forecasts."""
    from dataclasses import replace
    e = dfa.Engine(dev, replace(cfg0, fit_mode="stan"))
    grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]), device=dev)
    fit = e.fit(grid, Yd)
    fg = e.predict_grid(fit, fut)
    out = e.predict(fit, fg, n_samples=0, components=False)
    return out["yhat"][:, :fg.T].double().cpu().numpy()


def dropin(args, eng, keys, ds, Y, Yd, rank, world, bracket, max_over_ranks, sum_over_ranks,
           timed, parallel, device):
    """The reference's own entry points on this rank's series (pandas in,
    pandas out), timed with the headline's bracketing."""
    import tempfile
    import pandas as pd
    import distributed_forecasting_amd as dfa
    from distributed_forecasting_amd import diagnostics
    n = len(keys)
    T = len(ds)
    df = pd.DataFrame({"ds": np.tile(ds.astype("datetime64[ns]"), n),
                       "store": np.repeat(keys[:, 0], T).astype(np.int32),
                       "item": np.repeat(keys[:, 1], T).astype(np.int32),
                       "y": Y.reshape(-1)})
    steps = args.dropin_steps
    tot = sum_over_ranks(n)
    out = {}

    def fsi(cv=False):
        # df holds this rank's shard already
        r = dfa.forecast_store_items(df, device=int(device.index), cv_metrics=cv,
                                     return_metrics=cv)
        fr, met = r if cv else (r, None)
        if world > 1:
            fr = parallel.gather_frames(fr, device=device)
            if cv:
                import torch
                mt = torch.from_numpy(met[list(dfa.CV_METRICS)].to_numpy()).to(device)
                kt = torch.from_numpy(met[["store", "item"]].to_numpy(np.int64)).to(device)
                g = parallel.gather_results(kt, None, mt)
                met = g["metrics"]
        return fr, met
    el, ka, (fr, _) = timed(fsi, steps, warm=3, kernels=False)
    out["forecast_store_items"] = {
        "value": tot * steps / el, "unit": "series/s", "ms_per_call": el / steps * 1e3,
        "rows_out": int(len(fr)),
        "note": "groupBy('store','item').applyInPandas(forecast_store_item) equivalent "
                "(02_training.py:305-307): long pandas frame in (913k rows at 500 series), "
                "[ds, store, item, y, yhat, yhat_upper, yhat_lower] frame out (float32, int32 "
                "keys); grouping, grid bucketing, H2D/D2H and frame assembly included; N>1: "
                "this rank's hash shard + tensor all-gather of the frames"}
    el, ka, (fr, met) = timed(lambda: fsi(True), steps, warm=2)
    out["forecast_store_items_cv"] = {
        "value": tot * steps / el, "unit": "series/s", "ms_per_call": el / steps * 1e3,
        "kernels_ms": ka,
        "cv_metric_means": {k: float(np.nanmean(np.asarray(met[k] if hasattr(met, "columns") else
                                                           met[:, i].cpu().numpy())))
                            for i, k in enumerate(dfa.CV_METRICS[:4])},
        "note": "forecast_store_items(cv_metrics=True): the reference's train_model always runs "
                "cross_validation(horizon 90d, period 360d, initial 730d) + performance_metrics "
                "(02_training.py:178-188) — 3 fold refits + fold forecasts + K6 per bucket on "
                "the GPU, per-series mse/rmse/mae/mape returned (N>1: RCCL all-gather of the CV "
                "metrics with the keys)"}
    with tempfile.TemporaryDirectory() as tmp:
        store = dfa.ParamsStore(os.path.join(tmp, "params"), writer=f"r{rank}")
        dfa.forecast_store_items(df, params_store=store, device=int(device.index))
        model = dfa.ForecastStoreItemModel(store)
        futd = dfa.future_dates(ds, HORIZON)
        inp = pd.DataFrame({"ds": np.tile(futd.astype("datetime64[ns]"), n),
                            "store": np.repeat(keys[:, 0], len(futd)).astype(np.int32),
                            "item": np.repeat(keys[:, 1], len(futd)).astype(np.int32)})
        el, ka, _ = timed(lambda: model.predict(None, inp), steps, warm=3, kernels=False)
        out["pyfunc_predict"] = {
            "value": tot * steps / el, "unit": "series/s", "ms_per_call": el / steps * 1e3,
            "note": "ForecastStoreItemModel.predict(context, model_input) (model_wrapper.py:43-73) "
                    "from a params store: 1916 future+history rows per series, 1000-sample "
                    "intervals, no 0.5 s sleep"}
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))

    def cv_on():
        met = diagnostics.cv_metrics_device(eng, ds, Yd[:, :T], seasons=seasons)
        grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]),
                              device=int(device.index))
        fit = eng.fit(grid, Yd)
        fg = eng.predict_grid(fit, dfa.future_dates(ds, HORIZON))
        o = eng.predict(fit, fg, seed=0, components=False)
        if world > 1:
            # the exchange north_star names: keys, forecasts and the CV metrics
            blk = torch.stack([o["yhat"], o["yhat_lower"], o["yhat_upper"]], 1)
            parallel.gather_results(kd_local, blk, met[:, :4].contiguous(), fit.status)
        return met, o
    import torch
    kd_local = torch.from_numpy(keys.astype(np.int64)).to(device)
    el, ka, _ = timed(cv_on, steps)
    out["cv_on"] = {
        "value": tot * steps / el, "unit": "series/s", "ms_per_step": el / steps * 1e3,
        "kernels_ms": ka,
        "note": "train_model with its cross_validation(horizon='90 days', period='360 days', "
                "initial='730 days') + performance_metrics (02_training.py:178-188): 3 fold refits "
                "(1016/1376/1736 rows) + fold forecasts + K6, then the full fit + 90-day forecast "
                "with intervals; N>1: RCCL all-gather of keys, forecasts and the CV metrics; the "
                "headline value is the CV-off figure"}
    return out


def configs2(args, eng, ds, seasons, fut, rank, world, device, timed, sum_over_ranks, parallel, B,
             diagnostics, dfa):
    """BASELINE configs[2]: args.c2_series series in total, hash-sharded
    across the ranks (strong scaling): fit + forecast + metrics + all-gather."""
    from distributed_forecasting_amd import synthetic
    keys = keys_for(args.c2_series)
    mine = parallel.shard_indices(keys, rank, world) if world > 1 else np.arange(len(keys))
    T = len(ds)
    Y = synthetic.sales_matrix(len(keys), ds, config_index=2)[mine]
    Yd = torch_zeros_like_grid(Y, device)
    sid = torch_from(B.series_id(keys[mine]), device)
    kd = torch_from(keys[mine].astype(np.int64), device)
    counts = parallel.gather_counts(len(mine), device) if world > 1 else None

    def step():
        grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]),
                              device=int(device.index))
        fit = eng.fit(grid, Yd)
        fg = eng.predict_grid(fit, fut)
        out = eng.predict(fit, fg, seed=0, components=False, series_id=sid)
        met = diagnostics.insample_metrics(eng, Yd[:, :T], out["yhat"], out["yhat_lower"],
                                           out["yhat_upper"], mdape=False)
        if world > 1:
            import torch
            blk = torch.stack([out["yhat"], out["yhat_lower"], out["yhat_upper"]], 1)
            parallel.gather_results(kd, blk, met[:, :4].contiguous(), fit.status, counts=counts)
        return fit
    el, ka, fit = timed(step, args.c2_steps)
    tot = sum_over_ranks(len(mine))
    return {"value": tot * args.c2_steps / el, "unit": "series/s", "n_gpus": world,
            "steps": args.c2_steps, "ms_per_step": el / args.c2_steps * 1e3, "scaling": "strong",
            "series_total": tot, "series_per_rank": counts or [len(mine)], "kernels_ms": ka,
            "map_certified": float((fit.status == 70).float().mean().item()),
            "note": "configs[2]: 50k synthetic daily series x 1826 days (config_index 2) in total, "
                    "splitmix64((store << 32) | item) mod N shards, fit + 90-day forecast + "
                    "1000-sample intervals + metrics + RCCL all-gather per step"}


def ragged_leg(args, eng, device, timed, sum_over_ranks, B, dfa):
    """A staggered store-item table (each series its own launch date, two end
    dates: ~100 distinct date grids over 500 series) with inputs resident in
    HBM: one ragged launch per kernel (engine.RaggedGrid) vs one launch per
    distinct grid (the bucket path), each step = grids + fit + 90-day forecast
    with intervals."""
    import torch
    from distributed_forecasting_amd import engine as E, synthetic, training
    df = synthetic.staggered_frame(10, args.series_per_gpu // 10, n_starts=50, n_ends=2,
                                   max_delay_days=730)
    gkeys, rows = training.group_frame(df, ["store", "item"])
    ds_all = B.to_ns(df["ds"])
    y = df["y"].to_numpy(np.float64)
    bks = B.bucket_groups([ds_all[r] for r in rows], [y[r] for r in rows])
    packs = B.ragged_packs(bks, eng.config)
    assert len(packs) == 1
    cfg = eng.config
    dev = int(device.index)
    Tp = E.pad_rows(max(bk.fit_ds.shape[0] for bk in bks))
    sizes = [bk.Y.shape[0] for bk in bks]
    row0 = np.concatenate(([0], np.cumsum(sizes)))
    n = int(row0[-1])
    Yh = np.zeros((n, Tp))
    for j, bk in enumerate(bks):
        Yh[row0[j]:row0[j + 1], :bk.fit_ds.shape[0]] = bk.Y
    Yd = torch.from_numpy(Yh).to(device)
    pkeys = np.concatenate([gkeys[bk.members] for bk in bks])
    sid = torch.from_numpy(B.series_id(pkeys)).to(device)
    gof = np.repeat(np.arange(len(bks)), sizes)
    futs = [B.future_dates(bk.history_dates, HORIZON) for bk in bks]
    spec = []
    for bk in bks:
        f = bk.fit_ds
        spec.append((f, cfg.seasons(int(f[0]), int(f[-1]), B.min_positive_diff(f)), int(f[0]),
                     int(f[-1] - f[0])))

    def grid(j, T_pad=None):
        f, se, st, sc = spec[j]
        return dfa.build_grid(f, se, start_ns=st, t_scale_ns=sc, device=dev, T_pad=T_pad)

    fds = [s[0] for s in spec]
    st0 = [s[2] for s in spec]
    sc0 = [s[3] for s in spec]

    def one_launch():
        rg = E.RaggedGrid.build(fds, spec[0][1], st0, sc0, gof, device=dev, T_pad=Tp)
        fit = eng.fit(rg, Yd)
        fg = eng.predict_grid(fit, futs)
        return fit, eng.predict(fit, fg, seed=0, components=False, series_id=sid)

    def per_bucket():
        fits = []
        for j in range(len(bks)):
            sl = slice(int(row0[j]), int(row0[j + 1]))
            g = grid(j)
            Yj = torch.zeros((sizes[j], g.T_pad), dtype=torch.float64, device=device)
            Yj[:, :g.T] = Yd[sl, :g.T]
            fit = eng.fit(g, Yj)
            fg = eng.predict_grid(fit, futs[j])
            fits.append(eng.predict(fit, fg, seed=0, components=False, series_id=sid[sl]))
        return fits
    steps = args.dropin_steps
    el, ka, (fit, _) = timed(one_launch, steps)
    el_b, ka_b, _ = timed(per_bucket, steps)
    tot = sum_over_ranks(n)
    return {"value": tot * steps / el, "unit": "series/s", "ms_per_step": el / steps * 1e3,
            "kernels_ms": ka, "n_series": n, "n_grids": len(bks),
            "T_min": int(min(s[0].shape[0] for s in spec)), "T_max": int(Tp and max(s[0].shape[0] for s in spec)),
            "map_certified": float((fit.status == 70).float().mean().item()),
            "per_bucket_launches": {"value": tot * steps / el_b, "ms_per_step": el_b / steps * 1e3,
                                    "kernels_ms": ka_b},
            "note": "staggered table (synthetic.staggered_frame: 50 launch dates over 730 days, 2 "
                    "end dates): every kernel launched once for all grids (ragged) vs once per "
                    "distinct grid; inputs resident, grids + fit + forecast + intervals per step"}


def torch_zeros_like_grid(Y, device):
    import torch
    import distributed_forecasting_amd as dfa
    T = Y.shape[1]
    Yd = torch.zeros((Y.shape[0], dfa.pad_rows(T)), dtype=torch.float64, device=device)
    Yd[:, :T] = torch.from_numpy(Y).to(device)
    return Yd


def torch_from(a, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


if __name__ == "__main__":
    main()
