"""ForecastStep: the fit + forecast + metrics step captured into a hipGraph
and replayed.  Every kernel runs on every replay, so replay outputs must be
bitwise equal to the eager launches on the same inputs, and a replay after
set_inputs must equal an eager step on the new batch."""
import numpy as np
import pytest
import torch

import distributed_forecasting_amd as dfa
from distributed_forecasting_amd import batch as B, synthetic

pytestmark = pytest.mark.gpu


def _snap(r):
    o = {k: v.clone() for k, v in r["forecast"].items()}
    o["theta"] = r["fit"].theta.clone()
    o["f"] = r["fit"].f.clone()
    o["status"] = r["fit"].status.clone()
    o["metrics"] = r["metrics"].clone()
    return o


def _bits_equal(a, b):
    """Bitwise equality (NaN entries — the skipped MDAPE — compare equal)."""
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.dtype == torch.float64:
        return torch.equal(a.view(torch.int64), b.view(torch.int64))
    return torch.equal(a, b)


def test_graph_replay_equals_eager():
    ds = synthetic.daily_dates()
    n = 48
    Y1 = synthetic.sales_matrix(n, ds, config_index=1)
    Y2 = synthetic.sales_matrix(n, ds, config_index=3)
    keys = np.stack([np.ones(n, np.int64), np.arange(1, n + 1)], 1)
    sid = torch.from_numpy(B.series_id(keys)).cuda()
    eng = dfa.Engine(0)
    st = dfa.ForecastStep(eng, ds, n, series_id=sid)
    st.set_inputs(Y1)
    e1 = _snap(st.run())
    st.set_inputs(Y2)
    e2 = _snap(st.run())
    st.set_inputs(Y1)
    st.capture()
    r1 = _snap(st.replay())
    st.set_inputs(Y2)
    r2 = _snap(st.replay())
    torch.cuda.synchronize()
    Tf = st.Tf
    for e, r in ((e1, r1), (e2, r2)):
        for k in ("theta", "f", "status", "metrics"):
            assert _bits_equal(e[k], r[k]), k
        for k in ("yhat", "yhat_lower", "yhat_upper"):
            assert torch.equal(e[k][:, :Tf], r[k][:, :Tf]), k
    assert not torch.equal(r1["theta"], r2["theta"])
    assert bool((r2["status"] == 70).all())


@pytest.mark.parametrize("method", ["exact", "sample"])
def test_predict_parts_on_two_streams_equal_one_call(method):
    """pf_predict_args.parts: K4 on the current stream and K5 on a side
    stream give the same outputs as one call."""
    ds = synthetic.daily_dates("2015-01-01", "2017-12-31")
    n = 24
    Y = synthetic.sales_matrix(n, ds)
    eng = dfa.Engine(0)
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    fit = eng.fit(g, Yd)
    fg = eng.predict_grid(fit, dfa.future_dates(ds, 90))
    one = eng.predict(fit, fg, seed=5, interval_method=method)
    side = torch.cuda.Stream()
    two = eng.predict(fit, fg, seed=5, interval_method=method, mc_stream=side)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for k in one:
        assert torch.equal(one[k][:, :fg.T], two[k][:, :fg.T]), k
    # without trend bands K5 selects only the yhat tails: same intervals
    nc = eng.predict(fit, fg, seed=5, interval_method=method, components=False)
    for k in ("yhat", "yhat_lower", "yhat_upper"):
        assert torch.equal(one[k][:, :fg.T], nc[k][:, :fg.T]), k


def test_replay_after_a_larger_fit_on_the_same_engine():
    """A captured step keeps pointers into its context's fit workspace; a
    later, larger fit on the engine it was built from (shared per-device
    context) must not move that workspace under the graph."""
    ds = synthetic.daily_dates("2016-01-01", "2017-12-31")
    n = 16
    Y = synthetic.sales_matrix(n, ds)
    eng = dfa.Engine(0)
    st = dfa.ForecastStep(eng, ds, n)
    assert st.engine.ctx is not eng.ctx
    st.set_inputs(Y)
    e = _snap(st.run())
    st.capture()
    # a longer grid and a bigger batch on the shared context: its workspace grows
    big = synthetic.daily_dates()
    Yb = synthetic.sales_matrix(64, big)
    seasons = eng.config.seasons(int(big[0]), int(big[-1]), int(big[1] - big[0]))
    g = dfa.build_grid(big, seasons, start_ns=int(big[0]), t_scale_ns=int(big[-1] - big[0]))
    Yd = torch.zeros((64, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Yb).cuda()
    eng.fit(g, Yd)
    r = _snap(st.replay())
    torch.cuda.synchronize()
    for k in ("theta", "f", "status", "metrics"):
        assert _bits_equal(e[k], r[k]), k
    for k in ("yhat", "yhat_lower", "yhat_upper"):
        assert torch.equal(e[k][:, :st.Tf], r[k][:, :st.Tf]), k


def test_close_releases_the_private_context():
    """a step that made its own engine destroys that pf_ctx on
    close(); the shared per-device context and a caller-given private engine
    are left alone; a closed step cannot replay."""
    ds = synthetic.daily_dates("2016-01-01", "2017-12-31")
    n = 8
    Y = synthetic.sales_matrix(n, ds)
    eng = dfa.Engine(0)
    with dfa.ForecastStep(eng, ds, n) as st:
        st.set_inputs(Y)
        st.run()
        st.capture()
        st.replay()
        ctx = st.engine.ctx
        assert not ctx.closed
    assert ctx.closed and st.graph is None
    assert not eng.ctx.closed
    with pytest.raises(RuntimeError, match="capture"):
        st.replay()
    own = dfa.Engine(0, own_context=True)
    st2 = dfa.ForecastStep(own, ds, n)
    assert st2.engine is own
    st2.set_inputs(Y)
    st2.run()
    st2.close()
    assert not own.ctx.closed
    own.close()
    assert own.ctx.closed
    with pytest.raises(RuntimeError, match="shared"):
        eng.ctx.close()


def _cols_bits(t, T):
    t = t[..., :T].contiguous()
    if t.dtype == torch.float32:
        return t.view(torch.int32)
    if t.dtype == torch.float64:
        return t.view(torch.int64)
    return t


@pytest.mark.parametrize("components,metrics", [(False, "fast"), (False, True), (True, True)])
def test_fused_step_equals_separate_launches(components, metrics):
    """pf_fit_forecast's one launch (fit + K4 + K5 + K6 per workgroup) gives
    the bits of the separate fit / predict / metrics launches, eager and
    replayed, with and without the trend bands and components."""
    ds = synthetic.daily_dates()
    n = 40
    Y = synthetic.sales_matrix(n, ds, config_index=1)
    keys = np.stack([np.ones(n, np.int64), np.arange(1, n + 1)], 1)
    sid = torch.from_numpy(B.series_id(keys)).cuda()
    eng = dfa.Engine(0)
    snaps = {}
    for fuse in (True, False):
        st = dfa.ForecastStep(eng, ds, n, series_id=sid, components=components, metrics=metrics,
                              fuse=fuse)
        st.set_inputs(Y)
        r = st.run()
        torch.cuda.synchronize()
        assert st.fused is fuse
        Tf = st.Tf
        snap = {k: _cols_bits(v, Tf).clone() for k, v in r["forecast"].items()}
        snap.update(theta=_cols_bits(r["fit"].theta, 10 ** 6).clone(),
                    f=_cols_bits(r["fit"].f, 10 ** 6).clone(), status=r["fit"].status.clone(),
                    metrics=_cols_bits(r["metrics"], 10 ** 6).clone())
        snaps[fuse] = snap
        if fuse:
            st.capture()
            st.set_inputs(Y)
            r2 = st.replay()
            torch.cuda.synchronize()
            for k, v in r2["forecast"].items():
                assert torch.equal(_cols_bits(v, Tf), snap[k]), ("replay", k)
            assert torch.equal(_cols_bits(r2["metrics"], 10 ** 6), snap["metrics"])
        st.close()
    a, b = snaps[True], snaps[False]
    assert set(a) == set(b)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert (a["status"] == 70).all()


def test_fit_forecast_falls_back_and_reports():
    """Engine.fit_forecast: the fused call reports fused=True at a small
    batch; with only_fused on a layout it cannot fuse (sample intervals) it
    launches nothing; without only_fused it runs the parts."""
    ds = synthetic.daily_dates()
    n = 8
    Y = synthetic.sales_matrix(n, ds, config_index=1)
    eng = dfa.Engine(0)
    seasons = eng.config.seasons(int(ds[0]), int(ds[-1]), int(ds[1] - ds[0]))
    g = dfa.build_grid(ds, seasons, start_ns=int(ds[0]), t_scale_ns=int(ds[-1] - ds[0]))
    Yd = torch.zeros((n, g.T_pad), dtype=torch.float64, device="cuda")
    Yd[:, :g.T] = torch.from_numpy(Y).cuda()
    fg = dfa.build_grid(dfa.future_dates(ds, 90), seasons, start_ns=g.start_ns,
                        t_scale_ns=g.t_scale_ns, t_change=g.t_change)
    fit, out, met, fused = eng.fit_forecast(g, Yd, fg, components=False, metrics="fast")
    assert fused and met is not None and out["yhat"].shape[0] == n
    ref = eng.fit(g, Yd)
    o2 = eng.predict(ref, fg, components=False)
    torch.cuda.synchronize()
    T = fg.T
    assert torch.equal(_cols_bits(out["yhat_lower"], T), _cols_bits(o2["yhat_lower"], T))
    r = eng.fit_forecast(g, Yd, fg, interval_method="sample", only_fused=True)
    assert r == (None, None, None, False)
    fit3, out3, met3, fused3 = eng.fit_forecast(g, Yd, fg, interval_method="sample",
                                                components=False, metrics=True)
    torch.cuda.synchronize()
    assert not fused3 and met3 is not None
    assert torch.equal(_cols_bits(out3["yhat"], T), _cols_bits(o2["yhat"], T))


def test_fused_step_more_series_than_resident_workgroups():
    """1100 series (more workgroups than the GPU holds at once: the K5 work
    sharing's helpers must not wait while workgroups are still to start) —
    the fused launch still gives the separate launches' bits."""
    ds = synthetic.daily_dates("2016-01-01", "2017-12-30")
    n = 1100
    Y = synthetic.sales_matrix(n, ds, config_index=3)
    eng = dfa.Engine(0)
    snaps = {}
    for fuse in (True, False):
        st = dfa.ForecastStep(eng, ds, n, metrics="fast", fuse=fuse)
        st.set_inputs(Y)
        r = st.run()
        torch.cuda.synchronize()
        assert st.fused is fuse
        Tf = st.Tf
        snaps[fuse] = {k: _cols_bits(v, Tf).clone() for k, v in r["forecast"].items()}
        snaps[fuse]["metrics"] = _cols_bits(r["metrics"], 10 ** 6).clone()
        snaps[fuse]["theta"] = _cols_bits(r["fit"].theta, 10 ** 6).clone()
        st.close()
    for k in snaps[True]:
        assert torch.equal(snaps[True][k], snaps[False][k]), k
