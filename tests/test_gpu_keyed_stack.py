"""Parity of the keyed stack matcher (siddhi_amd/csrc/keyed_stack.hpp: k_ks_match + k_ks_order; opt-in with
SG_KEYED_STACK, measured slower than the tile matcher at config 4's density) against the oracle, bit for bit: every callback (one per trigger j, in arrival order), its
rows in ascending start order, timestamps and float bits.

The matcher keeps each key's open starts of `every e1=S[f1] -> e2=S[e2.x OP e1.x] within W` as a stack
(StreamPreStateProcessor.processAndReturn :363-403, expireEvents :325-361 restated per key); the order
pass sorts the records into callback order on the device.  Covered here: the four stack operators on float
(ties, NaN) and int values, chunked flushes that carry open starts, wide projections (start- and
trigger-side column reads), both entry formats, dense buckets that make rounds share keys and tasks
overflow their ring (the rerun kernel), a carried-only last task, and the device-resident flush."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _stack_matcher(monkeypatch):
    monkeypatch.setenv("SG_KEYED_STACK", "1")      # opt-in path (the tile matcher is the default)

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


def _pair(ql, k):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "keyed_followed_by"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _run(ql, d, k, ncols, chunk=None, flush_each=False, batch=True):
    o, g, ids = _pair(ql, k)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]],
              batch=batch, chunk=chunk, flush_each=flush_each)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


def _q(pattern, sel="e1.symbol, e2.price"):
    return synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') " \
        f"from {pattern} select {sel} insert into Out; end;"


@pytest.mark.parametrize("n,k,e", [(300_000, 20_000, 100), (1_000_000, 5_000, 20), (2_000_000, 200_000, 1000)])
def test_stack_matches_oracle(n, k, e):
    d = synth.stock_ticks(n, seed=synth.SEEDS[4] + 7, k=k, e=e)
    g = _run(synth.CONFIG4_QL, d, k, 2)
    assert g.kernel_ms("k_ks_match") > 0 and g.kernel_ms("k_ks_order") > 0


@pytest.mark.parametrize("op", ["<", "<=", ">=", ">"])
def test_stack_ops_float_ties_nan(op):
    d = synth.stock_ticks(400_000, seed=51, k=20_000, e=100)
    price = np.floor(d["price"] / np.float32(12)).astype(np.float32) * np.float32(12)
    price[::97] = np.float32("nan")
    d["price"] = price
    g = _run(_q(f"every e1=StockStream[price > 20] -> e2=StockStream[price {op} e1.price] within 1 sec"), d,
             20_000, 2)
    assert g.kernel_ms("k_ks_match") > 0


@pytest.mark.parametrize("op", [">", "<="])
def test_stack_ops_int(op):
    d = synth.stock_ticks(300_000, seed=52, k=20_000, e=50)
    d["volume"] = (d["volume"] % 7).astype(np.int32)
    g = _run(_q(f"every e1=StockStream[volume > 1] -> e2=StockStream[volume {op} e1.volume] within 2 sec",
                "e1.symbol, e2.volume"), d, 20_000, 2)
    assert g.kernel_ms("k_ks_match") > 0


def test_stack_chunked_flushes_carry_open_starts():
    d = synth.stock_ticks(400_000, seed=53, k=30_000, e=40)
    o, g, ids = _pair(synth.CONFIG4_QL, 30_000)
    paths = []
    cols = [ids[d["symbol"]], d["price"], d["volume"]]
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], cols, chunk=37_003, flush_each=True,
              after=lambda: paths.append((g.kernel_ms("k_ks_match") > 0, g.kernel_ms("ks_reject"))))
    compare_raw(o.raw_outputs(), g.raw_outputs(), 2)
    assert sum(p for p, _r in paths) >= len(paths) - 1, paths


def test_stack_wide_projection():
    """Start- and trigger-side column reads (e1.volume, e2.volume), the start's own price and a 5-word
    record (the general record writer and the general order copy)."""
    d = synth.stock_ticks(300_000, seed=54, k=25_000, e=60)
    g = _run(_q("every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 1 sec",
                "e1.symbol, e1.volume as v1, e2.price, e2.volume as v2, e1.price as p1"), d, 25_000, 5)
    assert g.kernel_ms("k_ks_match") > 0


def test_stack_16byte_entries(monkeypatch):
    monkeypatch.setenv("SG_KT_E16", "1")
    d = synth.stock_ticks(500_000, seed=55, k=20_000, e=50)
    g = _run(synth.CONFIG4_QL, d, 20_000, 2)
    assert g.kernel_ms("k_ks_match") > 0


@pytest.mark.parametrize("k,e", [(300, 1), (600, 2), (2_000, 4)])
def test_stack_dense_buckets_rerun(k, e, monkeypatch):
    """Few keys per bucket (forced past the heuristic): most rounds hold several events of one key, so the
    levels serialise them, and the ring of 1024 nodes overflows on windows holding more starts -- those
    tasks rerun with the larger ring."""
    monkeypatch.setenv("SG_KS_FORCE", "1")
    d = synth.stock_ticks(200_000, seed=56 + k, k=k, e=e)
    g = _run(synth.CONFIG4_QL, d, k, 2)
    assert g.kernel_ms("k_ks_match") > 0


def test_stack_falling_runs_rerun_for_many_completions(monkeypatch):
    """Long falling price runs per key: one trigger completes far more than KS_KS starts, which the first
    launch cannot stage, so its task reruns (up to KS_KS2 completions per trigger)."""
    monkeypatch.setenv("SG_KS_FORCE", "1")
    n, k = 200_000, 400
    d = synth.stock_ticks(n, seed=57, k=k, e=2)
    i = np.arange(n)
    # each key takes 20 consecutive events: 19 falling starts, then a price above all of them
    d["symbol"] = ((i // 20) % k).astype(d["symbol"].dtype)
    d["price"] = np.where(i % 20 == 19, np.float32(99.0), np.float32(90.0) - (i % 20).astype(np.float32))
    g = _run(synth.CONFIG4_QL, d, k, 2)
    assert g.kernel_ms("k_ks_match") > 0 and g.kernel_ms("ks_rerun_tasks") > 0


def test_stack_per_event_sends():
    d = synth.stock_ticks(30_000, seed=58, k=20_000, e=5)
    _run(synth.CONFIG4_QL, d, 20_000, 2, batch=False)


def test_stack_device_resident_matches_host_path():
    import torch
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    k, n = 50_000, 1_000_000
    d = synth.stock_ticks(n, seed=59, k=k, e=200)
    o, g, ids = _pair(synth.CONFIG4_QL, k)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]])
    gout = g.raw_outputs()
    compare_raw(o.raw_outputs(), gout, 2)
    g2 = GpuApp(synth.CONFIG4_QL)
    intern_symbols(g2, k)
    g2.start()
    ts = torch.from_numpy(d["ts"]).to(dev)
    sy = torch.from_numpy(ids[d["symbol"]].astype(np.int32)).to(dev)
    pr = torch.from_numpy(d["price"]).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    g2.push_device("StockStream", n, ts.data_ptr(), [sy.data_ptr(), pr.data_ptr(), 0], hip_stream=stream)
    g2.flush_device(hip_stream=stream)
    torch.cuda.synchronize()
    assert g2.kernel_ms("k_ks_match") > 0
    assert g2.match_count("query1") == int(np.sum(gout[0]["n_in"]))
