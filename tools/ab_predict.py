"""A/B of the forecast kernels between two engine builds (dev tool).

    python tools/ab_predict.py <lib_a.so> <lib_b.so> [out_dir]

Each library runs in its own process (the ctypes binding loads one library
per process): the same fits (linear, flat, logistic daily series, 730-day
history, 90-day horizon) and forecasts under both interval methods, with and
without trend bands / components, N = 1000 and 300 samples.  The parent
compares every output array bitwise and prints one JSON line per case."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(lib, out):
    from distributed_forecasting_amd import _lib
    _lib.load(os.path.abspath(lib))
    import torch
    import distributed_forecasting_amd as dfa
    from distributed_forecasting_amd import synthetic
    from distributed_forecasting_amd.engine import ProphetConfig

    dev = torch.device("cuda", 0)
    ds = synthetic.daily_dates("2016-01-01", "2017-12-30")
    n = 96
    Y = synthetic.sales_matrix(n, ds, config_index=3)
    fut = np.concatenate([ds, ds[-1] + synthetic.NS_PER_DAY * np.arange(1, 91)])
    res = {}
    for growth in ("linear", "flat", "logistic"):
        cfg = ProphetConfig.reference()
        cfg.growth = growth
        eng = dfa.Engine(0, cfg)
        seasons = cfg.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
        grid = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
        Yd = torch.zeros((n, grid.T_pad), dtype=torch.float64, device=dev)
        Yd[:, :len(ds)] = torch.from_numpy(Y).to(dev)
        cap = None
        if growth == "logistic":
            cap = torch.zeros_like(Yd)
            cap[:, :len(ds)] = 1.3 * Yd[:, :len(ds)].max(dim=1, keepdim=True).values
        fit = eng.fit(grid, Yd, cap=cap)
        fg = eng.predict_grid(fit, fut)
        cf = None if cap is None else cap[:, :1].expand(-1, fg.T_pad).contiguous()
        sid = torch.arange(n, dtype=torch.int32, device=dev)
        for method in ("sample", "exact"):
            for comp in (False, True):
                for ns in (1000, 300):
                    o = eng.predict(fit, fg, n_samples=ns, seed=7, components=comp, series_id=sid,
                                    interval_method=method, cap=cf)
                    for k, v in o.items():
                        res[f"{growth}/{method}/comp{int(comp)}/N{ns}/{k}"] = v[:, :fg.T].cpu().numpy()
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    la, lb = sys.argv[1], sys.argv[2]
    od = sys.argv[3] if len(sys.argv) > 3 else "/tmp"
    outs = []
    for tag, lib in (("a", la), ("b", lb)):
        p = os.path.join(od, f"ab_predict_{tag}.npz")
        subprocess.run([sys.executable, __file__, "--child", lib, p], check=True)
        outs.append(np.load(p))
    A, B = outs
    n_bad = 0
    for k in sorted(A.files):
        a, b = A[k], B[k]
        same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
        if not same:
            n_bad += 1
            d = float(np.nanmax(np.abs(a.astype(np.float64) - b))) if a.shape == b.shape else None
            print(json.dumps({"case": k, "bitwise_equal": False, "max_abs_diff": d}))
    print(json.dumps({"cases": len(A.files), "differ": n_bad}))
    sys.exit(1 if n_bad else 0)


if __name__ == "__main__":
    main()
