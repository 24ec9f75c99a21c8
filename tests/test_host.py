"""CPU: host-side logic of the drop-in layer (no kernel launches)."""
import os
import re
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import _lib, batch as B, diagnostics, synthetic, training
from distributed_forecasting_amd.engine import ProphetConfig, NS_PER_DAY
from oracle import prophet_oracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    """The C-ABI library loads and exports every function include/prophet_hip.h declares."""
    hdr = open(os.path.join(ROOT, "include", "prophet_hip.h")).read()
    decl = set(re.findall(r"^\s*(?:int|void|const char \*)\s*(pf_\w+)\s*\(", hdr, re.M))
    assert decl == set(_lib.EXPORTED)
    lib = _lib.load()
    for name in decl:
        assert hasattr(lib, name), name


def test_num_changepoints_host():
    for T, want in [(1826, 25), (730, 25), (10, 7), (2, 0), (31, 23), (32, 24), (33, 25)]:
        assert _lib.num_changepoints(T) == want
        assert len(po.changepoint_indices(T)) == want


def test_missing_library_fails_loudly():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from distributed_forecasting_amd import _lib\n"
            "try:\n    _lib.load('/nonexistent/libprophet_hip.so')\n"
            "except _lib.EngineUnavailable as e:\n    print('UNAVAILABLE')\n") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "UNAVAILABLE" in out.stdout


def test_build_id_matches_sources():
    """The in-tree library was compiled from the committed csrc/ + include/."""
    from distributed_forecasting_amd import build as bld
    bid = _lib.check_build_id()
    assert re.fullmatch(r"[0-9a-f]{32}", bid)
    assert _lib.load().pf_build_id().decode() == bid == bld.source_hash()


def test_stale_library_is_refused(tmp_path):
    """A .so whose sources changed after it was built is refused (not loaded)."""
    import shutil
    from distributed_forecasting_amd import build as bld
    csrc, inc = tmp_path / "csrc", tmp_path / "include"
    shutil.copytree(bld.CSRC, csrc)
    shutil.copytree(bld.INCLUDE, inc)
    so = tmp_path / "libprophet_hip.so"
    shutil.copy(bld.OUT, so)
    assert _lib.check_build_id(str(so), str(csrc), str(inc)) == bld.source_hash()
    with open(csrc / "pf_common.h", "a") as f:
        f.write("\n// edited after the build\n")
    with pytest.raises(_lib.EngineUnavailable, match="stale"):
        _lib.check_build_id(str(so), str(csrc), str(inc))
    # the same check guards load() of the in-tree path, in a fresh process
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from distributed_forecasting_amd import _lib, build\n"
            "build.CSRC = %r\n"
            "try:\n    _lib.load()\n"
            "except _lib.EngineUnavailable as e:\n    print('REFUSED', e)\n") % (ROOT, str(csrc))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "REFUSED" in out.stdout and "stale" in out.stdout, out.stdout + out.stderr


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    df = synthetic.store_item_frame(1, 1, "2017-01-01", "2017-03-01")
    with pytest.raises(RuntimeError, match="no GPU"):
        dfa.Prophet().fit(df[["ds", "y"]])


def test_logistic_requires_cap():
    # UPSTREAM setup_dataframe: raised before any GPU work
    df = synthetic.store_item_frame(1, 1, "2017-01-01", "2017-03-01")
    with pytest.raises(ValueError, match="Capacities must be supplied"):
        dfa.Prophet(growth="logistic").fit(df[["ds", "y"]])
    d2 = df[["ds", "y"]].assign(cap=100.0, floor=0.0)
    with pytest.raises(NotImplementedError, match="floor"):
        dfa.Prophet(growth="logistic").fit(d2)


def test_holiday_columns_match_oracle():
    """UPSTREAM make_holiday_features: window offsets, date matching of every
    hourly row of the day, '_delim_' keys sorted, same columns at predict."""
    import pandas as pd
    from distributed_forecasting_amd import holidays as H
    ds = synthetic.hourly_dates(n_hours=24 * 400)
    hd = pd.concat([H.synthetic_holidays([2016, 2017, 2018]),
                    pd.DataFrame({"holiday": ["xmas"], "ds": [pd.Timestamp("2016-12-25")],
                                  "lower_window": [-2], "upper_window": [1]})])
    spec = H.holiday_spec(hd, 10.0)
    X = H.holiday_columns(spec, ds)
    Xo, keys = po.holiday_features(ds, hd)
    assert list(spec.names) == keys and len(keys) == 14
    assert np.array_equal(X.T, Xo)
    assert "xmas_delim_-2" in keys and X.sum() > 0


def test_holiday_spec_errors():
    import pandas as pd
    from distributed_forecasting_amd import holidays as H
    hd = pd.DataFrame({"holiday": ["a", "a"], "ds": pd.to_datetime(["2016-01-01", "2017-01-01"]),
                       "prior_scale": [1.0, 2.0]})
    with pytest.raises(ValueError, match="consistent prior scale"):
        H.holiday_spec(hd)
    with pytest.raises(ValueError, match="both lower_window and upper_window"):
        H.holiday_spec(hd.drop(columns="prior_scale").assign(lower_window=0))


def test_allocate_forecasts():
    """02_training.py:235-247: ratios sales / SUM(sales) OVER (PARTITION BY
    item); y and yhat scaled; NaN future y stays NaN."""
    import pandas as pd
    sales = pd.DataFrame({"store": [1, 2, 1, 2], "item": [7, 7, 8, 8], "sales": [30.0, 10.0, 5.0, 5.0]})
    fc = pd.DataFrame({"ds": pd.to_datetime(["2018-01-01", "2018-01-02"] * 2), "item": [7, 7, 8, 8],
                       "y": [4.0, np.nan, 2.0, np.nan], "yhat": [8.0, 8.0, 2.0, 4.0]})
    out = dfa.allocate_forecasts(fc, sales, training_date=pd.Timestamp("2020-01-01"))
    assert list(out.columns) == ["date", "store", "item", "sales", "forecast", "training_date"]
    r = out[(out.store == 1) & (out.item == 7)].sort_values("date")
    assert np.allclose(r["forecast"], [6.0, 6.0]) and r["sales"].iloc[0] == 3.0 and np.isnan(r["sales"].iloc[1])
    r = out[(out.store == 2) & (out.item == 8)].sort_values("date")
    assert np.allclose(r["forecast"], [1.0, 2.0])
    assert len(out) == 8


def test_seasonality_auto_rules():
    cfg = ProphetConfig()
    d = NS_PER_DAY
    assert [s[0] for s in cfg.seasons(0, 1825 * d, d)] == ["yearly", "weekly"]
    assert [s[0] for s in cfg.seasons(0, 100 * d, d)] == ["weekly"]
    assert [s[0] for s in cfg.seasons(0, 10 * d, d)] == []
    assert [s[0] for s in cfg.seasons(0, 5 * d, 3600 * 10**9)] == ["daily"]
    assert [s[0] for s in cfg.seasons(0, 1825 * d, 7 * d)] == ["yearly"]
    ref = ProphetConfig.reference()
    assert ref.seasons(0, 100 * d, d) == [("yearly", 365.25, 10), ("weekly", 7.0, 3)]


def test_future_dates_daily():
    ds = synthetic.daily_dates()
    fut = B.future_dates(ds, 90)
    assert len(fut) == 1916
    assert np.array_equal(fut, po.make_future_dates(ds, 90))
    assert np.array_equal(fut[1826:] - ds[-1], NS_PER_DAY * np.arange(1, 91))


def test_bucket_groups_nan_and_signatures():
    ds = synthetic.daily_dates("2017-01-01", "2017-01-20")
    y1 = np.arange(20, dtype=float)
    y2 = y1 * 2
    y3 = y1.copy(); y3[5] = np.nan
    perm = np.random.default_rng(0).permutation(20)
    bks = B.bucket_groups([ds, ds[perm], ds], [y1, y2[perm], y3])
    assert len(bks) == 2
    b0 = [b for b in bks if len(b.members) == 2][0]
    assert b0.members.tolist() == [0, 1]
    assert np.array_equal(b0.Y[1], y2)             # sorted by ds
    b1 = [b for b in bks if len(b.members) == 1][0]
    assert len(b1.fit_ds) == 19 and len(b1.history_dates) == 20
    with pytest.raises(ValueError, match="less than 2 non-NaN"):
        B.bucket_groups([ds[:3]], [np.array([1.0, np.nan, np.nan])])


def test_group_frame_keeps_row_order():
    df = pd.DataFrame({"store": [2, 1, 2, 1, 2], "item": [1, 1, 1, 1, 1],
                       "ds": pd.date_range("2020-01-01", periods=5), "y": [5., 4., 3., 2., 1.]})
    keys, rows = training.group_frame(df, ["store", "item"])
    assert keys.tolist() == [[1, 1], [2, 1]]
    assert rows[0].tolist() == [1, 3] and rows[1].tolist() == [0, 2, 4]


def test_shard_hash_properties():
    keys = np.stack(np.meshgrid(np.arange(1, 11), np.arange(1, 51), indexing="ij"), -1).reshape(-1, 2)
    for G in (1, 2, 4, 8):
        sh = B.shard_of(keys, G)
        assert sh.min() >= 0 and sh.max() < G
        counts = np.bincount(sh, minlength=G)
        assert counts.sum() == 500
        if G > 1:
            assert counts.max() < 500 / G * 1.5
    # stable across calls and independent of the batch it is computed in
    assert np.array_equal(B.shard_of(keys[:7], 8), B.shard_of(keys, 8)[:7])
    sid = B.series_id(keys)
    assert sid.dtype == np.int32 and len(np.unique(sid)) == 500


def test_generate_cutoffs_matches_oracle():
    ds = synthetic.daily_dates()
    for h, i, p in [(90, 730, 360), (30, 365, 180), (90, 100, 45)]:
        a = diagnostics.generate_cutoffs(ds, h * NS_PER_DAY, i * NS_PER_DAY, p * NS_PER_DAY)
        b = po.generate_cutoffs(ds, h * NS_PER_DAY, i * NS_PER_DAY, p * NS_PER_DAY)
        assert a == b
    with pytest.raises(ValueError):
        diagnostics.generate_cutoffs(ds[:50], 90 * NS_PER_DAY, 730 * NS_PER_DAY, 360 * NS_PER_DAY)


def test_synthetic_shape_and_determinism():
    ds = synthetic.daily_dates()
    assert len(ds) == 1826
    a = synthetic.sales_matrix(3, ds)
    b = synthetic.sales_matrix(3, ds)
    assert np.array_equal(a, b) and a.min() >= 0 and np.all(a == np.round(a))
    df = synthetic.store_item_frame(2, 3)
    assert len(df) == 6 * 1826 and df["store"].dtype == np.int32


# ------------------------------------------------ hyperparameter search layout
def test_tuning_trials_and_layout():
    from distributed_forecasting_amd import tuning
    tr = tuning.sample_trials(64, seed=3)
    assert len(tr) == 64
    for t in tr:
        for k in tuning.PRIOR_KEYS:
            lo, hi = tuning.SEARCH_SPACE[k]
            assert np.exp(lo) <= t[k] <= np.exp(hi)
        assert t["seasonality_mode"] in ("additive", "multiplicative")
    assert tr == tuning.sample_trials(64, seed=3)
    lay = tuning.expand_trials(5, tr[:4], "multiplicative")
    seen = []
    for mode, (js, si, tj) in lay.items():
        assert all(tr[j]["seasonality_mode"] == mode for j in js)
        assert len(si) == len(tj) == 5 * len(js)
        assert np.array_equal(si[:5], np.arange(5)) and set(tj) == set(js)
        seen += js
    assert sorted(seen) == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        tuning.expand_trials(2, [dict(seasonality_mode="bogus")], "additive")


def test_prophet_json_record_layout():
    """serialize.json_to_record on a hand-built fbprophet-0.7.1-layout JSON
    (host only): theta order [k, m, delta, log sigma_obs, beta], time units,
    and the refusal of layouts the engine cannot serve."""
    import json
    from distributed_forecasting_amd import serialize
    d = {"mcmc_samples": 0, "y_scale": 12.5, "start": 1356998400.0, "t_scale": 86400.0 * 1825,
         "changepoints_t": [0.1, 0.5],
         "history_dates": pd.Series(pd.date_range("2013-01-01", periods=3), name="ds")
         .to_json(orient="split", date_format="iso"),
         "seasonalities": [["weekly"], {"weekly": {"period": 7, "fourier_order": 1,
                                                   "prior_scale": 10.0, "mode": "additive",
                                                   "condition_name": None}}],
         "extra_regressors": [[], {}],
         "params": {"k": [[0.3]], "m": [[0.6]], "delta": [[0.01, -0.02]],
                    "sigma_obs": [[0.05]], "beta": [[0.1, 0.2]]}}
    rec = serialize.json_to_record(json.dumps(d), keys=[1, 2])
    assert np.allclose(rec["theta"][0], [0.3, 0.6, 0.01, -0.02, np.log(0.05), 0.1, 0.2])
    assert rec["start_ns"] == 1356998400 * 10**9 and rec["t_scale_ns"] == 1825 * NS_PER_DAY
    assert rec["history_dates"][0] == pd.Timestamp("2013-01-01").value
    assert list(rec["season_orders"]) == [1] and rec["keys"].shape == (1, 2)
    t = np.linspace(0, 1, 5)
    tr = serialize._trend(d["params"], t, np.array(d["changepoints_t"]), "linear")
    want = [0.3 * x + 0.6 + sum(dl * (x - c) for dl, c in zip([0.01, -0.02], [0.1, 0.5]) if x >= c)
            for x in t]
    assert np.allclose(tr, want, rtol=0, atol=1e-15)
    bad = dict(d, params=dict(d["params"], beta=[[0.1, 0.2, 0.3]]))
    with pytest.raises(NotImplementedError, match="beyond the seasonal"):
        serialize.json_to_record(json.dumps(bad))
    with pytest.raises(NotImplementedError, match="mcmc"):
        serialize.json_to_record(json.dumps(dict(d, mcmc_samples=10)))


# ------------------------------------------------------------- params store
def _json_model(mode="additive", growth="linear"):
    import json
    d = {"mcmc_samples": 0, "y_scale": 12.5, "start": 1356998400.0, "t_scale": 86400.0 * 1825,
         "growth": growth, "seasonality_mode": mode, "interval_width": 0.95,
         "changepoints_t": [0.1, 0.5],
         "history_dates": pd.Series(pd.date_range("2013-01-01", periods=3), name="ds")
         .to_json(orient="split", date_format="iso"),
         "seasonalities": [["weekly"], {"weekly": {"period": 7, "fourier_order": 1,
                                                   "prior_scale": 10.0, "mode": mode,
                                                   "condition_name": None}}],
         "extra_regressors": [[], {}],
         "params": {"k": [[0.3]], "m": [[0.6]], "delta": [[0.01, -0.02]],
                    "sigma_obs": [[0.05]], "beta": [[0.1, 0.2]]}}
    return json.dumps(d)


def test_params_store_refuses_other_config(tmp_path):
    """an additive Prophet JSON imported into a store holding the
    reference (multiplicative) config is refused, not served as multiplicative;
    so is a different growth or interval width."""
    from distributed_forecasting_amd import serialize
    store = dfa.ParamsStore(str(tmp_path / "s"))          # reference config
    with pytest.raises(ValueError, match="seasonality_mode"):
        store.put_record(serialize.json_to_record(_json_model("additive"), keys=[1, 2]))
    with pytest.raises(ValueError, match="growth"):
        store.put_record(serialize.json_to_record(_json_model("multiplicative", "flat"), keys=[1, 2]))
    ok = serialize.json_to_record(_json_model("multiplicative"), keys=[1, 2])
    store.put_record(ok)
    assert len(store) == 1
    assert ok["series_id"][0] == B.series_id(np.array([[1, 2]]))[0]
    bad = dict(ok, interval_width=np.float64(0.8))
    with pytest.raises(ValueError, match="interval_width"):
        store.put_record(bad)
    with pytest.raises(ValueError, match="different ProphetConfig"):
        dfa.ParamsStore(str(tmp_path / "s"), config=ProphetConfig())
    d = __import__("json").loads(_json_model("multiplicative"))
    d["seasonalities"][1]["weekly"]["mode"] = "additive"
    with pytest.raises(NotImplementedError, match="own mode"):
        serialize.json_to_record(__import__("json").dumps(d))


def _writer(path, w, n):
    import numpy as np
    from distributed_forecasting_amd.serving import ParamsStore
    st = ParamsStore(path, writer=f"w{w}")
    for i in range(n):
        st.put_record({"keys": np.array([[w, i]], np.int64), "theta": np.zeros((1, 3))})


def test_params_store_concurrent_writers(tmp_path):
    """several writers on one directory (torchrun ranks / Spark
    executors) lose no record: names are unique per writer, the index is a
    directory scan."""
    import multiprocessing as mp
    path = str(tmp_path / "shared")
    dfa.ParamsStore(path)
    ctx = mp.get_context("fork")
    procs = [ctx.Process(target=_writer, args=(path, w, 12)) for w in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    st = dfa.ParamsStore(path)
    assert len(st.record_names()) == 48
    assert set(st.index()) == {(w, i) for w in range(4) for i in range(12)}
    # a refit written later wins
    st.put_record({"keys": np.array([[0, 0]], np.int64), "theta": np.ones((1, 3))})
    name, row = st.index()[(0, 0)]
    assert st.record(name)["theta"][row, 0] == 1.0


def test_holiday_record_roundtrip():
    from distributed_forecasting_amd import holidays as H
    hd = H.synthetic_holidays([2016, 2017], n_per_year=3)
    spec = H.holiday_spec(hd, 4.0, "additive")
    rec = B.holiday_record(spec)
    assert B.holiday_from_record(rec) == spec
    assert B.holiday_from_record({}) is None and B.holiday_record(None) == {}


def test_ragged_packs_group_by_layout():
    """Buckets share a ragged launch iff their auto seasonalities and
    changepoint counts agree (batch.ragged_packs)."""
    import numpy as np
    from distributed_forecasting_amd import batch as B, synthetic
    from distributed_forecasting_amd.engine import ProphetConfig
    ds = synthetic.daily_dates()
    y = np.arange(ds.shape[0], dtype=np.float64)
    parts = [(ds[s:], y[s:]) for s in (0, 30, 365)]          # >= 730 days: yearly on
    parts += [(ds[-400:], y[-400:]), (ds[-300:], y[-300:])]  # < 730 days: no yearly
    parts += [(ds[-20:], y[-20:])]                           # 20 rows: 15 changepoints
    bks = B.bucket_groups([p[0] for p in parts], [p[1] for p in parts])
    packs = B.ragged_packs(bks, ProphetConfig())              # auto seasonalities
    assert sorted(len(p) for p in packs) == [1, 2, 3], packs
    # the reference config forces yearly + weekly on: only the changepoint
    # count splits
    packs = B.ragged_packs(bks, ProphetConfig.reference())
    assert sorted(len(p) for p in packs) == [1, 5], packs


def test_group_frame_and_buckets_fast_paths():
    """group_frame's integer-code path (sorted input: no sort; shuffled input:
    one stable argsort) and bucket_groups' sorted fast path give the same
    groups, row order and buckets as the general path."""
    import numpy as np
    import pandas as pd
    from distributed_forecasting_amd import batch as B, synthetic, training
    df = synthetic.store_item_frame(3, 4, start="2016-01-01", end="2016-03-31")
    g0, r0 = training.group_frame(df, ["store", "item"])
    sh = df.sample(frac=1.0, random_state=1)
    g1, r1 = training.group_frame(sh, ["store", "item"])
    assert np.array_equal(g0, g1) and len(r0) == len(r1) == 12
    idx = sh.index.to_numpy()
    for a, b in zip(r1, r0):
        assert np.all(np.diff(a) > 0)                       # stable: input order kept
        assert np.array_equal(np.sort(idx[a]), b)
    # keys beyond the integer-code range take the lexsort path
    big = df.assign(store=df["store"].astype(np.int64) * (1 << 40))
    g2, r2 = training.group_frame(big, ["store", "item"])
    assert np.array_equal(g2[:, 1], g0[:, 1]) and all(np.array_equal(a, b) for a, b in zip(r2, r0))
    # buckets: sorted NaN-free groups (fast path) vs the same groups reversed
    ds = B.to_ns(df["ds"])
    y = df["y"].to_numpy(np.float64)
    fwd = B.bucket_groups([ds[r] for r in r0], [y[r] for r in r0])
    rev = B.bucket_groups([ds[r][::-1] for r in r0], [y[r][::-1] for r in r0])
    assert len(fwd) == len(rev) == 1
    assert np.array_equal(fwd[0].fit_ds, rev[0].fit_ds) and np.array_equal(fwd[0].Y, rev[0].Y)
    assert np.array_equal(fwd[0].members, rev[0].members)
    yn = [y[r].copy() for r in r0]
    yn[2][5] = np.nan
    mixed = B.bucket_groups([ds[r] for r in r0], yn)
    assert len(mixed) == 2 and sorted(len(b.members) for b in mixed) == [1, 11]
    assert pd.Series([b.fit_ds.shape[0] for b in mixed]).isin([90, 91]).all()


# ------------------------------------------------------ round-3 host additions
def test_dense_frame_fast_path_agrees_with_general_path():
    """training.dense_frame (the sorted sales table: no per-group work) gives
    the groups, dates and values group_frame + bucket_groups give, and
    declines every layout it does not cover."""
    df = synthetic.store_item_frame(3, 4, "2016-01-01", "2017-12-31")
    gk, ds0, Y = training.dense_frame(df, ["store", "item"])
    g1, rows = training.group_frame(df, ["store", "item"])
    ds = B.to_ns(df["ds"])
    y = df["y"].to_numpy(np.float64)
    bks = B.bucket_groups([ds[r] for r in rows], [y[r] for r in rows])
    assert len(bks) == 1 and np.array_equal(gk, g1)
    assert np.array_equal(ds0, bks[0].fit_ds) and np.array_equal(Y, bks[0].Y)
    assert np.shares_memory(Y, df["y"].to_numpy())          # a view, no copy
    _, _, none = training.dense_frame(df, ["store", "item"], value=None)
    assert none is None
    # declined: NaN y, shuffled groups, unequal lengths, different dates, unsorted dates
    d = df.copy()
    d.loc[5, "y"] = np.nan
    assert training.dense_frame(d, ["store", "item"]) is None
    assert training.dense_frame(df.iloc[::-1].reset_index(drop=True), ["store", "item"]) is None
    order = np.concatenate([np.arange(731, 2 * 731), np.arange(731), np.arange(2 * 731, len(df))])
    assert training.dense_frame(df.iloc[order].reset_index(drop=True), ["store", "item"]) is None
    assert training.dense_frame(df.iloc[1:].reset_index(drop=True), ["store", "item"]) is None
    d = df.copy()
    d.loc[731, "ds"] = d.loc[731, "ds"] - pd.Timedelta(days=1)
    assert training.dense_frame(d, ["store", "item"]) is None
    assert training.dense_frame(df.iloc[:0], ["store", "item"]) is None


def test_dense_guess_defers_only_the_row_checks():
    """training.dense_guess reads the layout off the first group; the layouts
    only the O(rows) checks can tell apart pass the guess and fail verify()
    (the callers then take the general path), the others fail the guess."""
    df = synthetic.store_item_frame(3, 4, "2016-01-01", "2017-12-31")
    gk, ds0, Y, verify = training.dense_guess(df, ["store", "item"])
    assert verify() and np.array_equal(gk, training.dense_frame(df, ["store", "item"])[0])
    T = len(ds0)
    late = []
    d = df.copy()
    d.loc[5 * T + 3, "y"] = np.nan                        # NaN in a later group
    late.append(d)
    d = df.copy()
    d.loc[4 * T + 7, "ds"] = d.loc[4 * T + 7, "ds"] + pd.Timedelta(hours=1)   # other dates
    late.append(d)
    d = df.copy()
    d.loc[3 * T + 2, "item"] = d.loc[3 * T + 2, "item"] + 1                  # key split
    late.append(d)
    for d in late:
        g = training.dense_guess(d, ["store", "item"])
        assert g is not None and not g[3]()
        assert training.dense_frame(d, ["store", "item"]) is None
    # caught by the guess itself: rows not a multiple of T, unsorted first
    # group, keys out of order
    assert training.dense_guess(df.iloc[:-1].reset_index(drop=True), ["store", "item"]) is None
    d = df.copy()
    d.loc[1, "ds"], d.loc[2, "ds"] = df.loc[2, "ds"], df.loc[1, "ds"]
    assert training.dense_guess(d, ["store", "item"]) is None
    order = np.concatenate([np.arange(T, 2 * T), np.arange(T), np.arange(2 * T, len(df))])
    assert training.dense_guess(df.iloc[order].reset_index(drop=True), ["store", "item"]) is None
    # one group: T = all rows
    one = df.iloc[:T].reset_index(drop=True)
    g = training.dense_guess(one, ["store", "item"])
    assert g[1].shape[0] == T and g[0].shape[0] == 1 and g[3]()


def _legacy_store(path, recs):
    """A params store in the first record format (manifest 'records' list of
    bucket_NNNNNN.npz files, no 'format' key)."""
    import json
    import os
    os.makedirs(path, exist_ok=True)
    names = []
    for i, rec in enumerate(recs):
        name = f"bucket_{i:06d}.npz"
        np.savez(os.path.join(path, name), **rec)
        names.append(name)
    with open(os.path.join(path, "manifest.json"), "w") as f:
        json.dump({"records": names, "config": ProphetConfig.reference().__dict__}, f)


def test_params_store_reads_format_1(tmp_path):
    """a store written by the previous code is indexed (its listed
    bucket records first, in manifest order), not silently empty; new records
    of the current format win for refitted keys."""
    from distributed_forecasting_amd import serialize
    r1 = serialize.json_to_record(_json_model("multiplicative"), keys=[1, 2])
    r2 = serialize.json_to_record(_json_model("multiplicative"), keys=[1, 3])
    r3 = dict(r1, keys=np.array([[1, 2]], np.int64))        # refit of (1, 2) in the old store
    path = str(tmp_path / "old")
    _legacy_store(path, [r1, r2, r3])
    st = dfa.ParamsStore(path)
    assert st.legacy_records == ["bucket_000000.npz", "bucket_000001.npz", "bucket_000002.npz"]
    idx = st.index()
    assert idx[(1, 2)] == ("bucket_000002.npz", 0) and idx[(1, 3)] == ("bucket_000001.npz", 0)
    name = st.put_record(dict(r2))
    assert st.index()[(1, 3)] == (name, 0) and len(st) == 2


def test_params_store_serving_fields_may_differ(tmp_path):
    """reopening a store with other serving-only settings
    (uncertainty_samples, interval_method, fit_mode) is allowed and those
    settings are the caller's; fit-defining fields must agree."""
    from dataclasses import replace
    path = str(tmp_path / "s")
    dfa.ParamsStore(path)
    cfg = replace(ProphetConfig.reference(), uncertainty_samples=200, interval_method="sample",
                  fit_mode="stan")
    st = dfa.ParamsStore(path, config=cfg)
    assert st.config.uncertainty_samples == 200 and st.config.fit_mode == "stan"
    with pytest.raises(ValueError, match="different ProphetConfig"):
        dfa.ParamsStore(path, config=replace(ProphetConfig.reference(), changepoint_prior_scale=0.5))
    with pytest.raises(ValueError, match="different ProphetConfig"):
        dfa.ParamsStore(path, config=replace(ProphetConfig.reference(), n_changepoints=10))


def test_params_store_generation_and_metrics(tmp_path):
    """A caller-given generation orders refits independently of wall clocks;
    metrics() returns the winning record's CV metrics per key."""
    from distributed_forecasting_amd import serialize
    st = dfa.ParamsStore(str(tmp_path / "s"), writer="a")
    other = dfa.ParamsStore(str(tmp_path / "s"), writer="b")
    rec = serialize.json_to_record(_json_model("multiplicative"), keys=[4, 5])
    m_new = np.arange(len(dfa.CV_METRICS), dtype=np.float64)[None, :]
    newer = dict(rec, cv_metrics=m_new, cv_metric_names=np.array(dfa.CV_METRICS))
    older = dict(rec, cv_metrics=m_new + 100, cv_metric_names=np.array(dfa.CV_METRICS))
    n2 = other.put_record(newer, generation=2)
    st.put_record(older, generation=1)                        # written later, older generation
    assert st.index()[(4, 5)] == (n2, 0)
    met = st.metrics()
    assert list(met.columns) == ["store", "item"] + list(dfa.CV_METRICS)
    assert met.shape[0] == 1 and met["mse"].iloc[0] == 0.0 and met["mdape"].iloc[0] == 6.0
    with pytest.raises(ValueError):
        st.put_record(rec, generation=-1)
