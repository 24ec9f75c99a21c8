"""Benchmark: series fit+forecast per second on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One step = the whole hot path for this rank's batch of series, inputs resident
in HBM: K1 design grid (history) -> prepare/init -> K3 fit (Stan L-BFGS warm-up
handed to the certified exact-MAP polish) -> K1 future grid -> K4/K5 90-day
forecast with 1000-sample 95% intervals (-> RCCL all-gather of the forecast
blocks when N>1).  Also timed in the same run and reported beside `value`:
`full_sampling` (every row's 1000 samples materialised) and `stan_full` (Stan's
full L-BFGS termination rules before the polish; same MAP).

Workload (N=1): BASELINE.json configs[1] — 500 synthetic Kaggle-shaped series
x 1826 days (SURVEY.md §8d generator).  N>1: weak scaling, 500 series per GPU
(10*N stores x 50 items) hash-sharded by (store, item).

roofline: the dominant kernel (k_fit), timed with HIP events recorded by the
engine on the launch stream.  Algorithmic FLOPs = the evaluations k_fit performed
(n_eval) x 4T(F+2C) per evaluation.
cpu_baseline: the CPU restatement (oracle/: Stan L-BFGS in C + numpy 1000-sample
predictive sampler), timed in a process pool on a bounded sample, rank 0, N=1.
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
FLOPS_PER_EVAL = 4 * T_DAYS * (26 + 2 * 25)      # 555,104
PEAK_FP64_TFLOPS = 78.6                            # MI355X FP64 matrix
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--series-per-gpu", type=int, default=SERIES_PER_GPU)
    ap.add_argument("--cpu-sample", type=int, default=384,
                    help="series in the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: min(16, cpu_count)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the full_sampling / stan_full timings (profiling runs)")
    return ap.parse_args()


# --------------------------------------------------------------- workload
def workload(world: int, per_gpu: int):
    from distributed_forecasting_amd import synthetic
    n_items = 50
    n_stores = max(1, (per_gpu * world + n_items - 1) // n_items)
    keys = np.stack(np.meshgrid(np.arange(1, n_stores + 1), np.arange(1, n_items + 1),
                                indexing="ij"), -1).reshape(-1, 2)[:per_gpu * world]
    ds = synthetic.daily_dates()
    Y = synthetic.sales_matrix(len(keys), ds, config_index=1)
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
    return out["yhat"]


def cpu_baseline(ds, Y, n_sample: int, workers: int):
    import multiprocessing as mp
    from oracle import stan_oracle as so
    so.lib()                                   # build/load the C oracle once
    jobs = [(ds, Y[i], 1000 + i) for i in range(n_sample)]
    ctx = mp.get_context("fork")               # no exec; runs before any GPU init
    with ctx.Pool(workers) as pool:
        pool.map(_cpu_one, jobs[:workers])     # warm the workers (imports)
        t0 = time.perf_counter()
        yh = pool.map(_cpu_one, jobs, chunksize=1)
        dt = time.perf_counter() - t0
    return n_sample / dt, dt, np.stack(yh)


def oracle_map_yhat(ds, Y, idx):
    from oracle import prophet_oracle as po, stan_oracle as so
    out = []
    for i in idx:
        st = po.build_problem(ds, Y[i])
        th = so.fit_map(st)[0]
        out.append(po.predict_point(st, po.params_from_theta(th, st.problem.S),
                                    po.make_future_dates(ds, HORIZON))["yhat"])
    return np.stack(out)


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
        workers = args.cpu_workers or min(16, os.cpu_count() or 1)
        n_s = max(args.cpu_sample, workers)
        rate, dt, cpu_yhat = cpu_baseline(ds, Y_all, n_s, workers)
        cpu = dict(value=rate, unit="series/s", cores=workers, kind="port",
                   sample=(f"first {n_s} of the {len(keys)} bench series; per series: Stan "
                           f"L-BFGS MAP (oracle C restatement) + 90-day forecast with "
                           f"{N_SAMPLES}-sample intervals (numpy restatement); "
                           f"{workers}-process pool, {dt:.1f} s wall"),
                   _yhat=cpu_yhat, _n=n_s)

    import torch
    import torch.distributed as dist
    import distributed_forecasting_amd as dfa
    from distributed_forecasting_amd import batch as B, parallel

    dev = local
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    mine = parallel.shard_indices(keys, rank, world) if world > 1 else np.arange(len(keys))
    n = len(mine)
    eng = dfa.Engine(dev)                       # reference config (02_training.py:162-169)
    cfg = eng.config
    seasons = cfg.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    Tp = dfa.pad_rows(len(ds))
    Yd = torch.zeros((n, Tp), dtype=torch.float64, device=f"cuda:{dev}")
    Yd[:, :len(ds)] = torch.from_numpy(Y_all[mine]).to(Yd.device)
    sid = torch.from_numpy(B.series_id(keys[mine])).to(Yd.device)
    fut = B.future_dates(ds, HORIZON)
    torch.cuda.synchronize()

    def step(method="exact", stan_faithful=False):
        grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]),
                              device=dev)
        fit = eng.fit(grid, Yd, stan_faithful=stan_faithful)
        fg = eng.predict_grid(fit, fut)
        out = eng.predict(fit, fg, seed=0, components=False, series_id=sid,
                          interval_method=method)
        if world > 1:
            blk = torch.stack([out["yhat"], out["yhat_lower"], out["yhat_upper"]], 1)
            parallel.gather_blocks(blk, counts=counts)
        return fit, fg, out

    counts = None
    if world > 1:
        cn = torch.tensor([n], device=Yd.device)
        allc = [torch.zeros_like(cn) for _ in range(world)]
        dist.all_gather(allc, cn)
        counts = [int(c.item()) for c in allc]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fit, fg, out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rec = eng.ctx.read_timings()
    eng.ctx.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=Yd.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([n], dtype=torch.int64, device=Yd.device)
        dist.all_reduce(tot)
        total_series = int(tot.item())
    else:
        total_series = n

    # per-kernel averages over the timed steps (HIP events on the launch stream)
    def averages(records):
        kern = {}
        for name, ms, grid_n in records:
            k = kern.setdefault(name, [0.0, 0, grid_n])
            k[0] += ms
            k[1] += 1
        return {k: v[0] / v[1] for k, v in kern.items()}
    kern_avg = averages(rec)

    def timed(**kw):
        """K more timed steps of a variant (same bracketing as the headline)."""
        step(**kw)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        eng.ctx.set_timing(True)
        t0_ = time.perf_counter()
        for _ in range(args.steps):
            step(**kw)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0_
        ka = averages(eng.ctx.read_timings())
        eng.ctx.set_timing(False)
        if world > 1:
            t_ = torch.tensor([el], dtype=torch.float64, device=Yd.device)
            dist.all_reduce(t_, op=dist.ReduceOp.MAX)
            el = float(t_.item())
        return el, ka

    # every row's intervals materialised from N samples (PF_INTERVAL_SAMPLE,
    # UPSTREAM's literal loop), and the reference-shaped optimizer run (Stan's
    # full L-BFGS termination rules before the polish)
    if args.no_variants:
        elapsed_s = elapsed_f = float("nan")
        kern_avg_s = kern_avg_f = {}
    else:
        elapsed_s, kern_avg_s = timed(method="sample")
        elapsed_f, kern_avg_f = timed(stan_faithful=True)

    # roofline of the dominant kernel (k_fit): algorithmic FLOPs = the
    # objective+gradient evaluations it performed (n_eval, L-BFGS only) x
    # 4T(F+2C) per evaluation
    with open(os.path.join(ROOT, "tests", "golden", "bench_manifest.json")) as f:
        man = json.load(f)
    E_all = np.array(man["E"], dtype=np.float64)
    E_mean = float(E_all.mean())
    evals = float(fit.n_eval.double().sum().item())
    fit_kernel = "k_fit_polish" if "k_fit_polish" in kern_avg else "k_fit"
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
    roof = {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic, "kernel": fit_kernel,
            "kernel_ms": kern_avg.get(fit_kernel), "flops_per_launch": flops_alg,
            "evals_algorithmic_per_launch": float(mine_E.sum()),
            "evals_performed_per_launch": evals,
            "achieved_performed": achieved_perf, "frac_performed": achieved_perf / PEAK_FP64_TFLOPS,
            "note": "FP64 (MI355X FP64 vector peak = FP64 matrix peak = 78.6 TF).  achieved = SURVEY "
                    "§8d algorithmic FLOPs (the oracle Stan run's evaluations E per series x "
                    "4T(F+2C)) / the fused fit+polish kernel's time; achieved_performed counts only "
                    "the L-BFGS evaluations the engine performed (its exact-MAP polish replaces "
                    "Stan's remaining ~260 evaluations/series); traffic = HBM bytes per launch "
                    "from rocprofv3 PMC (profiles/pmc_k_fit.json)"}
    # forecast kernel: HBM roofline of its algorithmic output bytes
    pred_bytes = 16.0 * len(fut) * n                # yhat, lo, hi, trend fp32 per row
    pred_s = (kern_avg.get("k_predict_det", float("nan")) +
              kern_avg.get("k_predict_mc", 0.0)) / 1e3

    value = total_series * args.steps / elapsed
    res = {
        "metric": "series fit+forecast/sec (1826d daily, 90d horizon, 1000-sample 95% intervals)",
        "value": value, "unit": "series/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md §8d Kaggle-shaped generator, seed 20261015+1)",
        "config": {"workload": "configs[1]: 500 series x 1826 days per GPU, Prophet MAP fit "
                               "(Stan L-BFGS warm-up + certified exact-MAP polish) + 90-day "
                               "forecast with "
                               "1000-sample 95% intervals (reference Prophet config, "
                               "02_training.py:162-169)",
                   "intervals": "exact: history rows (deterministic trend) draw the order "
                                "statistics of the 1000 noise samples exactly (same law); the "
                                "90 future rows materialise all 1000 samples",
                   "series_per_gpu": args.series_per_gpu, "series_total": total_series,
                   "series_this_rank": n, "T": len(ds), "horizon": HORIZON,
                   "uncertainty_samples": N_SAMPLES,
                   "parallelism": f"dp{world} (series hash-sharded by (store, item))"},
        "roofline": roof,
        "kernels_ms": kern_avg,
        "full_sampling": {"value": total_series * args.steps / elapsed_s, "unit": "series/s",
                          "ms_per_step": elapsed_s / args.steps * 1e3, "kernels_ms": kern_avg_s,
                          "note": "interval_method='sample': all 1916 rows x 1000 samples "
                                  "materialised per series (UPSTREAM's literal loop)"},
        "stan_full": {"value": total_series * args.steps / elapsed_f, "unit": "series/s",
                      "ms_per_step": elapsed_f / args.steps * 1e3, "kernels_ms": kern_avg_f,
                      "note": "stan_faithful=True: Stan's full L-BFGS termination rules (the "
                              "reference's optimizer run, ~350 evals/series) before the polish; "
                              "same MAP as the headline"},
        "forecast_roofline": {"bound": "hbm", "kernel": "k_predict_det + k_predict_mc",
                              "achieved": pred_bytes / pred_s / 1e9, "peak": PEAK_HBM_GBS,
                              "unit": "GB/s", "frac": pred_bytes / pred_s / 1e9 / PEAK_HBM_GBS,
                              "note": "algorithmic output bytes only; the kernel is "
                                      "VALU-bound (RNG + order statistics)"},
        "fit_stats": {"n_eval_mean": float(fit.n_eval.float().mean().item()),
                      "n_eval_max": int(fit.n_eval.max().item()),
                      "map_certified": float((fit.status == 70).float().mean().item()),
                      "E_oracle_stan_full_mean": E_mean},
        "cpu_baseline": None,
    }
    if cpu is not None:
        m = min(32, cpu.pop("_n"))
        cy = cpu.pop("_yhat")[:m]
        gy = out["yhat"][:m, :fg.T].double().cpu().numpy()
        ysc = np.abs(Y_all[:m]).max(1)
        my = oracle_map_yhat(ds, Y_all, range(m))
        res["accuracy"] = {
            "max_rel_dyhat_vs_oracle_map": float((np.abs(gy - my).max(1) / ysc).max()),
            "max_rel_dyhat_vs_oracle_stan_lbfgs": float((np.abs(gy - cy).max(1) / ysc).max()),
            "n_series": m,
            "note": "rel = max_t |yhat_gpu - yhat_oracle| / y_scale; the Stan-phase oracle "
                    "stops at Stan's tolerances (stall at the L1 kink), the MAP oracle is the "
                    "exact optimum the engine reaches"}
        res["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
