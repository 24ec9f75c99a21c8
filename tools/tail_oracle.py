"""The uncertified tail of a tools/bench_configs.py run:
for every series that ended without PF_ST_MAP (dumped with --tail), run the
oracle's Stan L-BFGS (C restatement, oracle/stan_lbfgs.c) on the same inputs
and compare the engine's returned objective with Stan's endpoint.

    python tools/tail_oracle.py gpurun_out/tail_c4.npz > profiles/..._tail.json

CPU only (runs in this container; the oracle is test infrastructure)."""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _one(args):
    cfgi, ds, y, cap = args
    from oracle import prophet_oracle as po, stan_oracle as so
    if cfgi == 5:
        import pandas as pd
        from distributed_forecasting_amd import holidays as H
        years = sorted(set(pd.to_datetime(ds).year)) + [int(pd.to_datetime(ds[-1]).year) + 1]
        hd = H.synthetic_holidays(years)
        cfg = dict(po.DEFAULT_CONFIG, growth="logistic")
        cfg["daily"] = (1.0, 4)
        st = po.build_problem(ds, y, cfg, cap=cap, holiday_cols_fn=lambda d: po.holiday_features(d, hd)[0])
    else:
        st = po.build_problem(ds, y)
    th, f, status, it, ne = so.fit_setup(st)
    thm, fm, *_ = so.polish(st.problem, th, 50, damp=True)
    return float(f), int(status), int(ne), float(fm)


def main():
    z = np.load(sys.argv[1], allow_pickle=False)
    cfgi = int(z["config"])
    n = len(z["index"])
    jobs = [(cfgi, z["ds"], z["y"][i], z["cap"][i] if cfgi == 5 else None) for i in range(n)]
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(_one, jobs)
    f_or = np.array([r[0] for r in res])
    f_map_or = np.array([r[3] for r in res])
    f = z["f"]
    rel = (f - f_or) / np.abs(f_or)
    rows = [{"index": int(z["index"][i]), "status": int(z["status"][i]), "n_eval": int(z["n_eval"][i]),
             "f": float(f[i]), "f_stan_engine": float(z["f_stan_engine"][i]),
             "f_oracle_stan": float(f_or[i]), "oracle_stan_status": res[i][1],
             "oracle_stan_n_eval": res[i][2], "f_oracle_polished": float(f_map_or[i]),
             "rel_f_minus_oracle_stan": float(rel[i])} for i in range(n)]
    print(json.dumps({"config_index": cfgi, "n": n,
                      "all_le_oracle_stan_plus_1e-6": bool(np.all(rel <= 1e-6)),
                      "max_rel_f_minus_oracle_stan": float(rel.max()),
                      "series": rows}))


if __name__ == "__main__":
    main()
