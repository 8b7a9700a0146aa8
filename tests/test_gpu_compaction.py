"""Long-running runtimes: after each flush the keyed followed-by, followed-by and window+aggregation paths
compact their buffers to what later flushes read (the open partials; the window content, carried in
per-group aggregator states).  Many flushes over a stream must give the oracle's output bit for bit while
`sg_query_buffered` stays bounded by the open state, not by the events ever pushed; the keyed tiles keep
taking later flushes (carried starts are a prefix that never triggers).
"""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


def _pair(ql, k, path):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == path, g.path("query1")
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _feed_flushing(o, g, stream, types, ts, cols, chunk, batch=True, after=None):
    """Chunks to both engines, the GPU runtime flushed after each; returns sg_query_buffered per flush."""
    si = o.L.or_stream_index(o.h, stream.encode())
    raw = raw_matrix(types, cols)
    held = []
    for s in range(0, len(ts), chunk):
        o.send_columns(si, ts[s:s + chunk], raw[s:s + chunk], None, batch)
        g.send_columns(stream, ts[s:s + chunk], [c[s:s + chunk] for c in cols], batch)
        g.flush()
        held.append(g.buffered("query1"))
        if after:
            after(s)
    return held


@pytest.mark.parametrize("e", [1, 10])
def test_keyed_many_flushes_stay_bounded_on_tiles(e):
    o, g, ids = _pair(synth.CONFIG4_QL, 2_000, "keyed_followed_by")
    n = 300_000
    d = synth.stock_ticks(n, seed=41, k=2_000, e=e)
    tiled = []
    held = _feed_flushing(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
                          20_011, after=lambda s: tiled.append(g.kernel_ms("k_kt_match") > 0 or
                                                               g.kernel_ms("k_kc_match") > 0))
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    win = 1_000 * e                                   # events per `within 1 sec`
    assert max(held) <= win + 1, held                 # the carried starts: open partials within W
    assert all(tiled), tiled                          # later flushes keep a device matcher (tiles / chunks)


def test_unkeyed_followed_by_many_flushes_stay_bounded():
    o, g, ids = _pair(synth.CONFIG1_QL, 50, "followed_by")
    n = 200_000
    d = synth.stock_ticks(n, seed=43, k=50, e=5)
    held = _feed_flushing(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
                          9_973)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    assert max(held) <= 5_000 + 1, held


WINDOWS = {
    "length_minmax": ("from StockStream[volume > 100]#window.length(37) select symbol, min(price) as lo, "
                      "max(price) as hi, count() as c group by symbol insert into Out;", 4, 60),
    "time_minmax": ("from StockStream[price > 20]#window.time(200) select symbol, min(price) as lo, "
                    "max(price) as hi, sum(volume) as sv group by symbol insert into Out;", 4, 2_000),
    "batch_group": ("from StockStream#window.lengthBatch(100) select symbol, sum(volume) as sv, "
                    "max(price) as mp group by symbol insert into Out;", 3, 200),
    "length_exact": ("from StockStream[price > 20]#window.length(1000) select symbol, avg(price) as ap, "
                     "sum(price) as sp, count() as c group by symbol insert into Out;", 4, 1_600),
}


@pytest.mark.parametrize("name", sorted(WINDOWS))
def test_window_agg_many_flushes_stay_bounded(name):
    sel, ncols, bound = WINDOWS[name]
    ql = "@app:playback " + synth.STOCK_STREAM + " @info(name='query1') " + sel
    o, g, ids = _pair(ql, 30, "window_agg")
    n = 60_000
    d = synth.stock_ticks(n, seed=47 + len(name), k=30, e=5)
    held = _feed_flushing(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
                          1_201)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    assert max(held) <= bound, held


def test_window_agg_exact_then_replay_rebuilds_the_states():
    """Sparse flushes take the exact tile path (the group states are not kept there); a dense stretch then
    needs the sequential replay, which rebuilds the states from the held window content.  Long values near
    2^40 make the dense windows' sums pass 2^53, so the replay's double arithmetic must match the
    reference's from the transition on."""
    ql = ("@app:playback define stream T (symbol string, price double, volume long); "
          "@info(name='query1') from T#window.time(1 sec) select symbol, sum(volume) as sv, avg(volume) as av, "
          "count() as c group by symbol insert into Out;")
    o, g, ids = _pair(ql, 7, "window_agg")
    r = synth.splitmix64(np.arange(130_000, dtype=np.uint64) + np.uint64(9))
    sparse = np.arange(30_000, dtype=np.int64)                       # 1 event / ms: windows of 1000
    dense = 30_000 + np.arange(100_000, dtype=np.int64) // 20        # 20 events / ms: windows of 20000
    ts = np.concatenate([sparse, dense]) + 1_000
    sym = ids[(r % np.uint64(7)).astype(np.int64)]
    vol = ((r >> np.uint64(8)) % np.uint64(1 << 39)).astype(np.int64) + (1 << 39)
    price = np.zeros(len(ts))
    kinds = []
    _feed_flushing(o, g, "T", ["STRING", "DOUBLE", "LONG"], ts, [sym, price, vol], 7_000,
                   after=lambda s: kinds.append("tile" if g.kernel_ms("k_wa_tile") > 0 else "seq"))
    compare_raw(o.raw_outputs(), g.raw_outputs(), 4)
    assert kinds[0] == "tile" and kinds[-1] == "seq", kinds


@pytest.mark.parametrize("ql,path,env", [
    (synth.CONFIG4_QL, "keyed_followed_by", None),
    (synth.CONFIG4_QL, "keyed_followed_by", "SG_KEYED_NO_TILES"),
    (synth.CONFIG1_QL, "followed_by", None),
])
def test_device_ingest_rejects_backwards_timestamps(ql, path, env, monkeypatch):
    """sg_push_device adopts HBM columns unchecked; the flush finds timestamps that go backwards (while the
    scatter / tile kernels stage them, or in one pass on the fallback pipelines) and fails loudly."""
    import torch
    from siddhi_amd.runtime import SiddhiGfxError
    if env:
        monkeypatch.setenv(env, "1")
    dev = torch.device("cuda:0")
    n = 200_000
    d = synth.stock_ticks(n, seed=5, k=100, e=10)
    for bad_at in (None, 123_457):
        g = GpuApp(ql)
        ids = intern_symbols(g, 100)
        g.add_query_callback("query1"); g.start()
        assert g.path("query1") == path
        ts = d["ts"].copy()
        if bad_at is not None:
            ts[bad_at] = ts[bad_at - 1] - 5
        t_ts = torch.from_numpy(ts).to(dev)
        t_sy = torch.from_numpy(ids[d["symbol"]]).to(dev)
        t_pr = torch.from_numpy(d["price"]).to(dev)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream(dev).cuda_stream
        g.push_device("StockStream", n, t_ts.data_ptr(), [t_sy.data_ptr(), t_pr.data_ptr(), 0], hip_stream=stream)
        if bad_at is None:
            g.flush_device(hip_stream=stream)
            assert g.match_count("query1") > 0
        else:
            with pytest.raises(SiddhiGfxError, match="backwards"):
                g.flush_device(hip_stream=stream)
        torch.cuda.synchronize()
