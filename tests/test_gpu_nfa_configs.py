"""BASELINE configs 3 and 5 (count/Kleene sequences, logical patterns) at synthetic scale on the device NFA
lanes (nfa.hip, one lane per partition key), against the oracle, bit for bit.

Config 3 is written literally (no `every`: each key's instance matches at most once, SURVEY §8 hazard 5,
SequenceTestCase.java:2165-2211) and in its `every` variant.  Config 5's logical half
(`every (e1 and e2) -> e3 within`) runs partitioned here; the full config-5 app (time window -> partitioned
logical + absent, with the Scheduler's one-instance-per-deadline order) is in test_gpu_partitioned_absent.py."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]

PART = synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') "

CONFIG3_LITERAL = PART + ("from e1=StockStream, e2=StockStream[price > e1.price]+, "
                          "e3=StockStream[price < e2[last].price] "
                          "select e1.symbol, e1.price as p1, e2[last].price as p2, e3.price as p3 "
                          "insert into Out; end;")
CONFIG3_EVERY = PART + ("from every e1=StockStream, e2=StockStream[price > e1.price]+, "
                        "e3=StockStream[price < e2[last].price] "
                        "select e1.symbol, e1.price as p1, e2[0].price as p2a, e2[last].price as p2, e3.price as p3 "
                        "insert into Out; end;")
CONFIG5_LOGICAL = PART + ("from every (e1=StockStream[price > 80] and e2=StockStream[volume > 900]) -> "
                          "e3=StockStream[price < 15] within 1 sec "
                          "select e1.symbol, e1.price as p1, e2.volume as v2, e3.price as p3 insert into Out; end;")
CONFIG5_OR = PART + ("from every (e1=StockStream[price > 95] or e2=StockStream[volume > 990]) -> "
                     "e3=StockStream[price < 12] within 500 milliseconds "
                     "select e1.price as p1, e2.volume as v2, e3.price as p3 insert into Out; end;")


def _run(ql, n, seed, k, e, ncols, chunk=None):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    d = synth.stock_ticks(n, seed=seed, k=k, e=e)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], chunk=chunk)
    oo, go = o.raw_outputs(), g.raw_outputs()
    compare_raw(oo, go, ncols)
    return int(np.sum(go[0]["n_in"]))


@pytest.mark.parametrize("n,k", [(40_000, 200), (200_000, 1000)])
def test_config3_literal_sequence(n, k):
    rows = _run(CONFIG3_LITERAL, n, synth.SEEDS[3], k, 1, 4)
    assert 0 < rows <= k                                   # at most one match per key


@pytest.mark.parametrize("n,k,chunk", [(40_000, 200, None), (100_000, 1000, 33_333)])
def test_config3_every_sequence(n, k, chunk):
    assert _run(CONFIG3_EVERY, n, synth.SEEDS[3], k, 1, 5, chunk=chunk) > 0


@pytest.mark.parametrize("n,k,e", [(60_000, 300, 2), (200_000, 2000, 20)])
def test_config5_partitioned_logical_and(n, k, e):
    assert _run(CONFIG5_LOGICAL, n, synth.SEEDS[5], k, e, 4) > 0


def test_config5_partitioned_logical_or():
    assert _run(CONFIG5_OR, 60_000, synth.SEEDS[5] + 1, 300, 2, 3) > 0
