"""CPU diagnostic (oracle only): where along Stan's L-BFGS trajectory does a
series commit to the basin its full run's polish reaches?  For the series the
GPU's default fit put in a worse basin (tools/diag_basin_floor.py output) and
a sample of other series: Stan L-BFGS stopped after k iterations (k on a
grid), the exact-MAP polish from there, and the objective / relative decrease
profile of the trajectory.
    python tools/diag_basin_commit.py gpurun_out/r04a_basin_floor.json [n_normal] [out.json]"""
import json
import os
import sys
from multiprocessing import Pool

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from distributed_forecasting_amd import synthetic
from oracle import prophet_oracle as po, stan_oracle as so

KS = [10, 20, 30, 40, 50, 60, 70, 80, 90, 100, 120, 140, 160, 180, 200, 250, 300, 400, 10000]
SEEDS = {"config_index=1": dict(config_index=1), "config_index=2": dict(config_index=2),
         "seed=1001": dict(seed=1001), "seed=1002": dict(seed=1002)}


def one(job):
    seed_name, s, n, tag = job
    ds = synthetic.daily_dates()
    Y = synthetic.sales_matrix(n, ds, **SEEDS[seed_name])
    st = po.build_problem(ds, Y[s])
    pb = st.problem
    rows = []
    for k in KS:
        th, f, status, it, ne = so.lbfgs(pb, st.theta0, so.default_opts(max_iter=k))
        thp, fp, nn, _, _, cert = so.polish(pb, th, 50, damp=True, return_cert=True)
        rows.append(dict(k=k, it=it, n_eval=ne, status=status, f=f, f_pol=fp, cert=cert,
                         dtheta=float(np.max(np.abs(thp - th)))))
        if status != 40:     # converged before the cap: later caps give the same run
            break
    return dict(seed=seed_name, s=s, tag=tag, rows=rows)


def main():
    src = json.load(open(sys.argv[1]))
    n_norm = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    out = sys.argv[3] if len(sys.argv) > 3 else None
    n = src["n"]
    jobs = []
    rng = np.random.default_rng(0)
    for name, r in src["seeds"].items():
        for v in r["map_violators"]:
            jobs.append((name, v["s"], n, "violator"))
        for s in rng.choice(n, n_norm // len(src["seeds"]), replace=False):
            jobs.append((name, int(s), n, "normal"))
    with Pool(min(8, os.cpu_count() or 1)) as p:
        res = p.map(one, jobs, chunksize=1)
    for r in res:
        fb = min(x["f_pol"] for x in r["rows"])
        r["f_best"] = fb
        prof = []
        for x in r["rows"]:
            prof.append(f'k={x["k"]}:{(x["f_pol"] - fb) / abs(fb):.1e}')
        print(r["tag"], r["seed"], r["s"], "n_eval_full", r["rows"][-1]["n_eval"], " ".join(prof), flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
