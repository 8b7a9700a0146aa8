"""Parity of the keyed followed-by path (SG_PATH_KEYED_FOLLOWED_BY, config 4 of BASELINE.json:
`partition with (symbol of StockStream)` around the config-1 pattern) against the oracle, which
restates the per-key partition instances (PartitionStreamReceiver / PartitionRuntimeImpl).

These tests pin the bucketed-tile matcher (keyed_tiles.hpp) with its device trigger-order pass (k_kt_order,
keyed_order.hpp) and the key-sort pipelines (SG_KEYED_NO_CHUNKS: the chunk-sorted pipeline that takes carry-free
flushes by default has its own file, test_gpu_keyed_chunks.py); the opt-in stack matcher has its own file,
test_gpu_keyed_stack.py."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _tile_matcher(monkeypatch):
    monkeypatch.delenv("SG_KEYED_STACK", raising=False)
    monkeypatch.setenv("SG_KEYED_NO_CHUNKS", "1")

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


def _pair(ql, k):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "keyed_followed_by"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _run(ql, n, seed, k, e, ncols, chunk=None, flush_each=False, batch=True):
    o, g, ids = _pair(ql, k)
    d = synth.stock_ticks(n, seed=seed, k=k, e=e)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
              batch=batch, chunk=chunk, flush_each=flush_each)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


@pytest.mark.parametrize("n,k,e", [(20_000, 50, 1), (300_000, 20_000, 100), (200_000, 1000, 10),
                                   (1_000_000, 5_000, 100)])
def test_config4_matches_oracle(n, k, e):
    """Bucketed-tile pipeline (keyed_tiles.hpp): one flush over a resident stream, records put in callback
    order on the device (k_kt_order)."""
    g = _run(synth.CONFIG4_QL, n, synth.SEEDS[4], k, e, 2)
    assert g.kernel_ms("k_kt_match") > 0 and g.kernel_ms("k_kt_order") > 0


@pytest.mark.parametrize("n,k,e", [(300_000, 20_000, 100), (1_000_000, 5_000, 100)])
def test_config4_host_ordered_records(n, k, e, monkeypatch):
    """Without the device order pass (SG_KT_NO_ORDER) the records are sorted by trigger with hipcub at
    materialisation: the same callbacks."""
    monkeypatch.setenv("SG_KT_NO_ORDER", "1")
    g = _run(synth.CONFIG4_QL, n, synth.SEEDS[4], k, e, 2)
    assert g.kernel_ms("k_kt_match") > 0 and g.kernel_ms("k_kt_order") < 0


@pytest.mark.parametrize("n,k,e", [(20_000, 50, 1), (1_000_000, 5_000, 100)])
def test_config4_16byte_entries(n, k, e, monkeypatch):
    """The 16-B entry format (kept for relative timestamps wider than 21 bits), forced by its test hook."""
    monkeypatch.setenv("SG_KT_E16", "1")
    g = _run(synth.CONFIG4_QL, n, synth.SEEDS[4], k, e, 2)
    assert g.kernel_ms("k_kt_match") > 0


def test_config4_wide_timestamps_use_16byte_entries():
    """2.2M ticks at 1 event/ms span more than 2^21 ms: the 16-B format is chosen on its own."""
    g = _run(synth.CONFIG4_QL, 2_200_000, 29, 20_000, 1, 2)
    assert g.kernel_ms("k_kt_match") > 0


@pytest.mark.parametrize("tile,chunk", [("4096", "4096"), ("2048", "4096"), ("2048", "8192")])
def test_config4_tile_variants(tile, chunk, monkeypatch):
    """The other matcher tile / scatter chunk instantiations (tuning hooks) on a multi-tile stream."""
    monkeypatch.setenv("SG_KT_TILE", tile)
    monkeypatch.setenv("SG_KT_CHUNK", chunk)
    g = _run(synth.CONFIG4_QL, 1_000_000, 28, 5_000, 100, 2)
    assert g.kernel_ms("k_kt_match") > 0


@pytest.mark.parametrize("n,k,e", [(20_000, 50, 1), (300_000, 20_000, 100)])
def test_config4_sort_pipeline_matches_oracle(n, k, e, monkeypatch):
    """The packed key-sort pipeline on the same streams (it takes flushes the tiles cannot)."""
    monkeypatch.setenv("SG_KEYED_NO_TILES", "1")
    g = _run(synth.CONFIG4_QL, n, synth.SEEDS[4], k, e, 2)
    assert g.kernel_ms("k_kf_scan") > 0


def test_config4_dense_window_falls_back_from_tiles():
    """4 keys at 1000 events/ms: one key's `within` window holds ~250k events, far more than a tile's
    back-halo, so the matcher raises its overflow flag and the sort pipeline re-runs the flush."""
    g = _run(synth.CONFIG4_QL, 60_000, 27, 4, 1000, 2)
    assert g.kernel_ms("k_kt_match") < 0 and g.kernel_ms("k_kf_scan") > 0


def test_config4_chunked_flushes_carry_open_starts():
    _run(synth.CONFIG4_QL, 120_000, 21, 3000, 20, 2, chunk=9_973, flush_each=True)


def test_config4_per_event_sends():
    _run(synth.CONFIG4_QL, 4_000, 22, 40, 1, 2, batch=False)


@pytest.mark.parametrize("pattern,sel,ncols", [
    ("every e1=StockStream[volume > 200] -> e2=StockStream[price < e1.price]", "e1.symbol as s, e1.volume as v, e2.price as p", 3),
    ("every e1=StockStream -> e2=StockStream[volume > e1.volume and price > 30]", "e1.price as a, e2.volume as b", 2),
    ("every e1=StockStream[price > 50] -> e2=StockStream[price > e1.price] within 40 milliseconds",
     "e2.price - e1.price as d, e1.volume * 2 as v", 2),
])
def test_keyed_variants(pattern, sel, ncols):
    ql = synth.STOCK_STREAM + f" partition with (symbol of StockStream) begin @info(name='query1') from {pattern} " \
                              f"select {sel} insert into Out; end;"
    _run(ql, 100_000, 23, 500, 5, ncols, chunk=25_000, flush_each=True)


def test_keyed_int_partition_key():
    ql = synth.STOCK_STREAM + " partition with (volume of StockStream) begin @info(name='query1') " \
                              "from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 1 sec " \
                              "select e1.symbol, e2.price, e2.volume insert into Out; end;"
    _run(ql, 100_000, 24, 100, 2, 3)


def test_config4_general_pipeline_matches_packed(monkeypatch):
    """The index-gather pipeline (used when the payload cannot be packed into the sort) on the same
    chunked stream as the packed one."""
    monkeypatch.setenv("SG_KEYED_NO_PACK", "1")
    _run(synth.CONFIG4_QL, 120_000, 25, 3000, 20, 2, chunk=9_973, flush_each=True)


def test_keyed_long_key_uses_general_pipeline():
    ql = ("define stream T (k long, price float, v int); partition with (k of T) begin @info(name='query1') "
          "from every e1=T[price > 20] -> e2=T[price > e1.price] within 50 milliseconds "
          "select e1.k as k, e2.price as p, e1.v as v insert into Out; end;")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "keyed_followed_by"
    n = 60_000
    d = synth.stock_ticks(n, seed=26, k=700, e=4)
    key = d["symbol"].astype(np.int64) * np.int64(1_000_003) - np.int64(1 << 40)
    feed_both(o, g, "T", ["LONG", "FLOAT", "INT"], d["ts"], [key, d["price"], d["volume"]], chunk=15_000)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 3)


def _run_data(ql, d, k, ncols):
    o, g, ids = _pair(ql, k)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]])
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


@pytest.mark.parametrize("op", ["<", "<=", ">=", "==", "!="])
def test_tiled_compare_ops_float_ties_nan(op):
    """The matcher's trigger-centric walk (kt_back) summarises the events between a start and a trigger per
    operator; prices quantised to 8 values (ties) with NaNs sprinkled in, over several tiles per bucket."""
    d = synth.stock_ticks(400_000, seed=31, k=3_000, e=100)
    price = np.floor(d["price"] / np.float32(12)).astype(np.float32) * np.float32(12)
    price[::97] = np.float32("nan")
    d["price"] = price
    ql = synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') " \
        f"from every e1=StockStream[price > 20] -> e2=StockStream[price {op} e1.price] within 1 sec " \
        "select e1.symbol, e2.price insert into Out; end;"
    g = _run_data(ql, d, 3_000, 2)
    assert g.kernel_ms("k_kt_match") > 0


@pytest.mark.parametrize("op", [">", "<=", "==", "!="])
def test_tiled_compare_ops_int(op):
    d = synth.stock_ticks(300_000, seed=32, k=2_000, e=50)
    d["volume"] = (d["volume"] % 7).astype(np.int32)
    ql = synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') " \
        f"from every e1=StockStream[volume > 1] -> e2=StockStream[volume {op} e1.volume] within 2 sec " \
        "select e1.symbol, e2.volume insert into Out; end;"
    g = _run_data(ql, d, 2_000, 2)
    assert g.kernel_ms("k_kt_match") > 0


@pytest.mark.parametrize("tile", ["2048", "4096"])
def test_tiled_wide_projection_owner_writes(tile, monkeypatch):
    """Records wider than 4 words (start- and trigger-side column gathers) are written by the two entries'
    owner lanes straight into the tile's record slab (no LDS staging)."""
    monkeypatch.setenv("SG_KT_TILE", tile)
    d = synth.stock_ticks(300_000, seed=33, k=2_500, e=60)
    ql = synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') " \
        "from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 1 sec " \
        "select e1.symbol, e1.volume as v1, e2.price, e2.volume as v2, e1.price as p1 insert into Out; end;"
    g = _run_data(ql, d, 2_500, 5)
    assert g.kernel_ms("k_kt_match") > 0


@pytest.mark.parametrize("keybits", [21, 22])
@pytest.mark.parametrize("e16", [False, True])
def test_config4_wide_key_space_many_buckets(keybits, e16, monkeypatch):
    """Integer partition keys spread over 2^21 / 2^22 values need pb = 11 / 12 bucket bits: the scatter's
    dynamic LDS then exceeds the 64 KiB default and is raised with hipFuncSetAttribute (both entry
    formats).  The keys are drawn from a small pool so that keys repeat and matches exist."""
    if e16:
        monkeypatch.setenv("SG_KT_E16", "1")
    ql = ("define stream StockStream (symbol string, price float, volume int); "
          "partition with (volume of StockStream) begin @info(name='query1') "
          "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
          "select e1.volume, e2.price insert into Out; end;")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "keyed_followed_by"
    ids_o, ids_g = intern_symbols(o, 4), intern_symbols(g, 4)
    assert np.array_equal(ids_o, ids_g)
    n = 400_000
    d = synth.stock_ticks(n, seed=31 + keybits, k=4, e=100)
    rng = np.random.default_rng(keybits)
    pool = rng.integers(0, 1 << keybits, 20_000, dtype=np.int64)
    pool[0] = (1 << keybits) - 1
    vol = pool[rng.integers(0, len(pool), n)].astype(np.int32)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids_g[d["symbol"]], d["price"], vol])
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    assert g.kernel_ms("k_kt_match") > 0
