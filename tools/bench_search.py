"""Batched hyperparameter search throughput, 1 GPU, JSON line.

  python tools/bench_search.py [n_series] [n_trials]

n synthetic Kaggle-shaped series x 1826 days, M trials drawn from the AutoML
search space (notebooks/automl/...:111-117: prior scales loguniform,
seasonality mode additive/multiplicative).  Each (series, trial) pair is
scored by UPSTREAM-cutoff cross-validation (horizon 90 d, period 360 d,
initial 730 d: three refits of 1016 / 1376 / 1736 rows + 90-day forecasts +
smape via K6), all pairs of one mode batched into the same launches; then
every series is refit on its full history with its best trial.  One untimed
warm-up search on a few series, then the whole search timed.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=500)
    ap.add_argument("trials", type=int, nargs="?", default=8)
    args = ap.parse_args()
    import torch
    from distributed_forecasting_amd import synthetic, tuning

    ds = synthetic.daily_dates()
    Y = synthetic.sales_matrix(args.n, ds, config_index=1)
    Yd = torch.from_numpy(Y).cuda()
    trials = tuning.sample_trials(args.trials, seed=7)
    tuning.hyperparameter_search(0, ds, Yd[:8], trials).best_fit(0, ds, Yd[:8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = tuning.hyperparameter_search(0, ds, Yd, trials)
    fits = res.best_fit(0, ds, Yd)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    col = list(tuning.L.CV_METRICS).index("smape")
    st = np.concatenate([fb.fit.status.cpu().numpy() for _, fb in fits.values()])
    print(json.dumps({
        "metric": "hyperparameter search: (series x trial) CV evaluations/sec",
        "value": args.n * args.trials / dt, "unit": "series-trials/s",
        "series_per_s": args.n / dt, "seconds": dt, "n_series": args.n, "n_trials": args.trials,
        "modes": sorted({t["seasonality_mode"] for t in trials}),
        "best_smape_mean": float(np.nanmean(res.metrics[np.arange(args.n), res.best_trial, col])),
        "best_refit_map_certified": float(np.mean(st == 70)),
        "work_per_pair": "3 CV refits (1016/1376/1736 rows) + 3 x 90-day point forecasts + "
                         "smape (K6); per series: + 1 full-history refit with the best trial",
    }))


if __name__ == "__main__":
    main()
