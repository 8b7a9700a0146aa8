"""Parity of the window + aggregation path (SG_PATH_WINDOW_AGG, config 2 of BASELINE.json) against the
oracle: bit-exact rows, timestamps and callback grouping, including the double-valued avg/sum.

The exact fast path (k_wa_tile) and the sequential general path (k_wa_seq) are both covered: float
prices that are multiples of 2^-S go through the fixed-point tile kernel; min/max and arbitrary doubles
go through the per-group replay of the reference's arithmetic.
"""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


def _pair(ql, k):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "window_agg"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _stock(n, seed, k, e=1):
    d = synth.stock_ticks(n, seed=seed, k=k, e=e)
    return d


def _run_stock(ql, n, seed, k, ncols, batch=True, chunk=None, flush_each=False, e=1):
    o, g, ids = _pair(ql, k)
    d = _stock(n, seed, k, e)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
              batch=batch, chunk=chunk, flush_each=flush_each)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


@pytest.mark.parametrize("n,k", [(20_000, 10), (200_000, 1000)])
def test_config2_matches_oracle(n, k):
    g = _run_stock(synth.CONFIG2_QL, n, synth.SEEDS[2], k, 4)
    assert g.kernel_ms("k_wa_tile") > 0     # the exact fast path ran


def test_config2_per_event_sends():
    _run_stock(synth.CONFIG2_QL, 5_000, 3, 20, 4, batch=False)


def test_config2_chunked_flushes_keep_window_history():
    _run_stock(synth.CONFIG2_QL, 60_000, 5, 50, 4, chunk=7_001, flush_each=True)


def test_config2_small_chunks_batch_selection():
    _run_stock(synth.CONFIG2_QL, 30_000, 8, 30, 4, chunk=97)


@pytest.mark.parametrize("sel,ncols", [
    ("select symbol, min(price) as lo, max(price) as hi, count() as c group by symbol", 4),
    ("select max(volume) as hv, sum(volume) as sv, avg(volume) as av", 3),
    ("select symbol, price, volume", 3),
    ("select symbol, sum(volume) as sv, avg(price) as ap group by symbol", 3),
])
def test_window_selector_variants(sel, ncols):
    ql = synth.STOCK_STREAM + f" @info(name='query1') from StockStream[volume > 100]#window.length(37) {sel} " \
                              "insert into Out;"
    _run_stock(ql, 40_000, 13, 25, ncols, chunk=1_000)


def test_window_inexact_doubles_use_exact_replay():
    """Arbitrary doubles: the fixed-point check fails, the sequential replay must still be bit-exact."""
    ql = ("define stream T (symbol string, price double, volume long); "
          "@info(name='query1') from T[price > 0.25]#window.length(100) select symbol, sum(price) as s, "
          "avg(price) as a, count() as c, min(price) as lo group by symbol insert into Out;")
    o, g, ids = _pair(ql, 40)
    n = 30_000
    r = synth.splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(77))
    price = (r >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    sym = ids[(r % np.uint64(40)).astype(np.int64)]
    vol = (r % np.uint64(1000)).astype(np.int64)
    ts = np.arange(n, dtype=np.int64) + 1_000
    feed_both(o, g, "T", ["STRING", "DOUBLE", "LONG"], ts, [sym, price, vol], chunk=2_500)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 5)
    assert g.kernel_ms("k_wa_seq") > 0


def test_window_long_sums():
    ql = ("define stream T (k int, v long); "
          "@info(name='query1') from T#window.length(500) select k, sum(v) as s, avg(v) as a, max(v) as m "
          "group by k insert into Out;")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    n = 50_000
    r = synth.splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(5))
    k = (r % np.uint64(17)).astype(np.int32)
    v = ((r >> np.uint64(20)) % np.uint64(1 << 30)).astype(np.int64) - (1 << 29)
    ts = np.arange(n, dtype=np.int64)
    feed_both(o, g, "T", ["INT", "LONG"], ts, [k, v], chunk=4_000)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 4)


# ---- #window.time (TimeWindowProcessor) and #window.lengthBatch (LengthBatchWindowProcessor) ----

def _run_app(ql, n, seed, k, ncols, e, batch=True, chunk=None, flush_each=False):
    o, g, ids = _pair(ql, k)
    d = _stock(n, seed, k, e)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
              batch=batch, chunk=chunk, flush_each=flush_each)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


TIME_QL = ("@app:playback " + synth.STOCK_STREAM +
           " @info(name='query1') from StockStream[price > 20]#window.time({T}) {sel} insert into Out;")


@pytest.mark.parametrize("t,e,batch,chunk", [(50, 3, False, None), (1000, 2, True, 997), (7, 1, True, 31)])
def test_time_window_exact_path(t, e, batch, chunk):
    """Playback clock: per-event sends (now = each event's ts) and batches (now = the batch's last ts)."""
    ql = TIME_QL.format(T=t, sel="select symbol, avg(price) as ap, sum(price) as sp, count() as c group by symbol")
    g = _run_app(ql, 30_000, 31, 40, 4, e, batch=batch, chunk=chunk)
    assert g.kernel_ms("k_wa_tile") > 0


def test_time_window_replay_min_max_chunked_flushes():
    ql = TIME_QL.format(T=200, sel="select symbol, min(price) as lo, max(price) as hi, sum(volume) as sv "
                                   "group by symbol")
    _run_app(ql, 20_000, 32, 15, 4, 5, chunk=1_234, flush_each=True)


def test_time_window_wider_than_a_tile_halo_uses_replay():
    """20k events per window: the LDS halo of the exact tile path cannot hold it."""
    ql = TIME_QL.format(T=1000, sel="select symbol, avg(price) as ap, count() as c group by symbol")
    g = _run_app(ql, 60_000, 36, 40, 3, 20, chunk=4_999)
    assert g.kernel_ms("k_wa_seq") > 0


def test_time_window_no_group_and_plain_projection():
    _run_app(TIME_QL.format(T=30, sel="select avg(price) as ap, count() as c"), 10_000, 33, 20, 2, 2, chunk=500)
    _run_app(TIME_QL.format(T=30, sel="select symbol, price"), 5_000, 34, 20, 2, 2, chunk=500)


BATCH_QL = synth.STOCK_STREAM + " @info(name='query1') from StockStream[price > 20]#window.lengthBatch({L}) {sel} " \
                                "insert into Out;"


@pytest.mark.parametrize("sel,ncols", [
    ("select symbol, sum(price) as sp, count() as c group by symbol", 3),
    ("select symbol, min(price) as lo, max(volume) as hv, avg(volume) as av group by symbol", 4),
    ("select sum(volume) as sv, count() as c", 2),
    ("select symbol, price, volume", 3),
])
def test_length_batch_window(sel, ncols):
    """Batches span send chunks and flushes; with group-by the batch's RESET (a copy of its first event)
    resets only that event's group."""
    _run_app(BATCH_QL.format(L=97, sel=sel), 20_000, 35, 12, ncols, 1, chunk=1_500, flush_each=True)
