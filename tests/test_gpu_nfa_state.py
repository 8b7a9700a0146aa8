"""The NFA's pattern state against the oracle's, in the shape of the reference's
StreamPreStateProcessor.StreamPreState.snapshot (StreamPreStateProcessor.java:450-469): after every flush, per
partition instance (creation order) and pre-state processor (the parser's preStateProcessors order), the
initialized flag, the pending and new-and-every StateEvent lists -- each StateEvent's timestamp, type and slot
event chains (timestamps and attribute values) -- and an absent processor's lastScheduledTime must equal the
restatement's (sg_query_state_json vs or_query_state_json).  This is the state a snapshot carries
(tests/test_gpu_snapshot.py checks the round trip), compared field for field rather than through outputs."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import intern_symbols, raw_matrix
from test_gpu_nfa_configs import CONFIG3_EVERY, CONFIG3_LITERAL, CONFIG5_LOGICAL, PART

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]

SHAPES = {
    "config3_every": (CONFIG3_EVERY, 30_000, 60, False),
    "config3_literal": (CONFIG3_LITERAL, 30_000, 60, False),
    "config5_logical": (CONFIG5_LOGICAL, 30_000, 80, False),
    "pattern_within": (PART + "from every e1=StockStream[price > 30] -> e2=StockStream[price > e1.price]<2:4> -> "
                       "e3=StockStream[price < e2[last].price] within 2 sec select e1.symbol, e1.price as p1, "
                       "e3.price as p3 insert into Out; end;", 30_000, 60, False),
    "partitioned_absent": ("@app:playback " + synth.STOCK_STREAM + " partition with (symbol of StockStream) begin "
                           "@info(name='query1') from every e1=StockStream[price > 80] -> "
                           "not StockStream[volume > 990] for 3 sec select e1.symbol, e1.price insert into Out; end;",
                           30_000, 40, True),
    "unpartitioned_sequence": (synth.STOCK_STREAM + "@info(name='query1') from every e1=StockStream, "
                               "e2=StockStream[price > e1.price]+, e3=StockStream[price < e2[last].price] "
                               "select e1.price as p1, e3.price as p3 insert into Out;", 20_000, 20, False),
}


@pytest.mark.parametrize("name", sorted(SHAPES))
def test_pattern_state_matches_oracle(name):
    ql, n, k, rr = SHAPES[name]
    d = synth.stock_ticks_rr(n, 3, k) if rr else synth.stock_ticks(n, seed=17, k=k, e=1)
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    si = o.L.or_stream_index(o.h, b"StockStream")
    cols = [gi[d["symbol"]], d["price"], d["volume"]]
    raw = raw_matrix(STOCK_TYPES, cols)
    checked = 0
    # an early cut too: a non-every sequence completes once per partition, so only its first events leave partials
    for lo, hi in ((0, 50), (50, n // 5), (n // 5, n // 2), (n // 2, n)):
        o.send_columns(si, d["ts"][lo:hi], raw[lo:hi], None, False)
        g.send_columns("StockStream", d["ts"][lo:hi], [c[lo:hi] for c in cols], False)
        g.raw_outputs()                                      # flush
        want, got = o.state_map("query1"), g.state_map("query1")
        assert len(got["instances"]) == len(want["instances"])
        for gi_, wi in zip(got["instances"], want["instances"]):
            assert gi_ == wi, (name, lo, gi_["key"])
        checked += sum(len(p["pending"]) + len(p["new_and_every"]) for inst in want["instances"]
                       for p in inst["processors"])
    assert checked > 0                                       # the cut points hold live partial matches
