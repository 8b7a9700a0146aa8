"""Parity of the chunk-sorted keyed pipeline (keyed_chunks.hpp: k_kc_sort -> k_kc_slices -> k_kc_match -> the
trigger-order pass in slice mode), which takes every keyed followed-by flush without carried starts -- the
bench's device-resident step -- against the oracle (per-key partition instances, PartitionStreamReceiver /
PartitionRuntimeImpl restated), bit for bit: rows, timestamps and callback grouping.

The scenarios are those of test_gpu_keyed.py for the bucketed tiles: densities from 1 to 100 events per ms,
several slices and buckets, ties and NaNs under every comparison, integer keys, wide records, wide key spaces,
carried starts handed to the next flush (which the bucketed tiles take), and the fallbacks (a chunk spanning
512 ms or more, a dense window)."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


@pytest.fixture(autouse=True)
def _chunk_pipeline(monkeypatch):
    monkeypatch.delenv("SG_KEYED_STACK", raising=False)
    monkeypatch.delenv("SG_KEYED_NO_CHUNKS", raising=False)


def _pair(ql, k):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "keyed_followed_by"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _run_data(ql, d, k, ncols, **kw):
    o, g, ids = _pair(ql, k)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]], **kw)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


def _keyed(pattern, sel):
    return synth.STOCK_STREAM + f" partition with (symbol of StockStream) begin @info(name='query1') from {pattern} " \
                                f"select {sel} insert into Out; end;"


@pytest.mark.parametrize("n,k,e", [(100_000, 5_000, 40), (300_000, 20_000, 100), (400_000, 1000, 40),
                                   (1_000_000, 5_000, 100), (3_000_000, 100_000, 1000)])
def test_config4_chunks_match_oracle(n, k, e):
    d = synth.stock_ticks(n, seed=synth.SEEDS[4], k=k, e=e)
    g = _run_data(synth.CONFIG4_QL, d, k, 2)
    assert g.kernel_ms("k_kc_match") > 0 and g.kernel_ms("k_kt_order") > 0


def test_config4_chunks_then_carried_flushes():
    """The first flush (no carried starts) runs the chunks; its carried starts go to the bucketed tiles of the
    next flushes."""
    d = synth.stock_ticks(300_000, seed=21, k=3000, e=40)
    _run_data(synth.CONFIG4_QL, d, 3000, 2, chunk=100_003, flush_each=True)


def test_config4_wide_chunk_falls_back():
    """At 10 events per ms an 8192-event chunk spans 819 ms (more than the 8-bit chunk-relative timestamps): the
    bucketed tiles take the flush."""
    d = synth.stock_ticks(200_000, seed=8, k=3000, e=10)
    g = _run_data(synth.CONFIG4_QL, d, 3000, 2)
    assert g.kernel_ms("k_kc_match") < 0 and g.kernel_ms("k_kt_match") > 0


def test_config4_skewed_buckets_fall_back():
    """Keys drawn from a small pool leave some buckets with more than a slice's T triggers: the matcher raises
    the overflow flag and another pipeline (the bucketed tiles, or the key sort when a falling run completes more
    than KT_MAXREC starts at one trigger) re-runs the flush."""
    ql = ("define stream StockStream (symbol string, price float, volume int); "
          "partition with (volume of StockStream) begin @info(name='query1') "
          "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
          "select e1.volume, e2.price insert into Out; end;")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    ids_g = intern_symbols(g, 4)
    intern_symbols(o, 4)
    n = 400_000
    d = synth.stock_ticks(n, seed=43, k=4, e=100)
    rng = np.random.default_rng(43)
    pool = rng.integers(0, 1 << 12, 300, dtype=np.int64)
    vol = pool[rng.integers(0, len(pool), n)].astype(np.int32)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids_g[d["symbol"]], d["price"], vol])
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    assert g.kernel_ms("k_kc_match") < 0


@pytest.mark.parametrize("op", ["<", "<=", ">=", "==", "!=", ">"])
def test_chunks_compare_ops_float_ties_nan(op):
    d = synth.stock_ticks(400_000, seed=31, k=3_000, e=100)
    price = np.floor(d["price"] / np.float32(12)).astype(np.float32) * np.float32(12)
    price[::97] = np.float32("nan")
    d["price"] = price
    ql = _keyed(f"every e1=StockStream[price > 20] -> e2=StockStream[price {op} e1.price] within 1 sec",
                "e1.symbol, e2.price")
    g = _run_data(ql, d, 3_000, 2)
    assert g.kernel_ms("k_kc_match") > 0


@pytest.mark.parametrize("op", [">", "<=", "==", "!="])
def test_chunks_compare_ops_int(op):
    d = synth.stock_ticks(300_000, seed=32, k=2_000, e=50)
    d["volume"] = (d["volume"] % 7).astype(np.int32)
    ql = _keyed(f"every e1=StockStream[volume > 1] -> e2=StockStream[volume {op} e1.volume] within 2 sec",
                "e1.symbol, e2.volume")
    g = _run_data(ql, d, 2_000, 2)
    assert g.kernel_ms("k_kc_match") > 0


def test_chunks_wide_projection():
    d = synth.stock_ticks(300_000, seed=33, k=2_500, e=60)
    ql = _keyed("every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 1 sec",
                "e1.symbol, e1.volume as v1, e2.price, e2.volume as v2, e1.price as p1")
    g = _run_data(ql, d, 2_500, 5)
    assert g.kernel_ms("k_kc_match") > 0


@pytest.mark.parametrize("pattern,sel,ncols", [
    ("every e1=StockStream[volume > 200] -> e2=StockStream[price < e1.price] within 500 milliseconds",
     "e1.symbol as s, e1.volume as v, e2.price as p", 3),
    ("every e1=StockStream[price > 50] -> e2=StockStream[price > e1.price] within 40 milliseconds",
     "e1.symbol as s, e2.price as p", 2),
])
def test_chunks_keyed_variants(pattern, sel, ncols):
    d = synth.stock_ticks(400_000, seed=23, k=500, e=50)
    g = _run_data(_keyed(pattern, sel), d, 500, ncols)
    assert g.kernel_ms("k_kc_match") > 0


@pytest.mark.parametrize("keybits", [12, 21])
def test_chunks_integer_keys(keybits):
    """Integer partition keys: few buckets (pb = 2) and a wide key space (pb = 11)."""
    ql = ("define stream StockStream (symbol string, price float, volume int); "
          "partition with (volume of StockStream) begin @info(name='query1') "
          "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
          "select e1.volume, e2.price insert into Out; end;")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    ids_o, ids_g = intern_symbols(o, 4), intern_symbols(g, 4)
    n = 400_000
    d = synth.stock_ticks(n, seed=31 + keybits, k=4, e=100)
    rng = np.random.default_rng(keybits)
    # (12 bits: every key value, so that buckets are even -- a skewed bucket overflows its slice and the flush
    # goes to the bucketed tiles, test_config4_skewed_buckets_fall_back)
    pool = rng.integers(0, 1 << keybits, 20_000, dtype=np.int64) if keybits > 12 else np.arange(1 << keybits)
    pool[0] = (1 << keybits) - 1
    vol = pool[rng.integers(0, len(pool), n)].astype(np.int32)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids_g[d["symbol"]], d["price"], vol])
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    assert g.kernel_ms("k_kc_match") > 0


def test_chunks_per_event_sends():
    d = synth.stock_ticks(30_000, seed=22, k=40, e=50)
    g = _run_data(synth.CONFIG4_QL, d, 40, 2, batch=False)
    assert g.kernel_ms("k_kc_match") > 0
