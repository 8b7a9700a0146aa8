"""Null attribute values through the C ABI (sg_batch.nulls): the NFA and general single-stream paths load
them (null compares false, CompareConditionExpressionExecutor.java:38-41; arithmetic on null is null; a
null projects as null; aggregators skip null arguments), bit-exact against the oracle.  The scan paths
refuse a batch with nulls (SG_E_UNSUPPORTED) instead of computing a different result."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd.runtime import GpuApp, SiddhiGfxError

pytestmark = pytest.mark.gpu

S = "define stream S (symbol string, price float, volume int);"


def _events(n, seed, p_null=0.15):
    rng = np.random.default_rng(seed)
    syms = ["A", "B", "C", None]
    ev = []
    for i in range(n):
        sym = syms[int(rng.integers(0, 4))] if rng.random() < p_null else syms[int(rng.integers(0, 3))]
        price = None if rng.random() < p_null else float(np.float32(rng.integers(0, 10000) / 100))
        vol = None if rng.random() < p_null else int(rng.integers(0, 1000))
        ev.append((1000 + i * 3, [sym, price, vol]))
    return ev


def _both(ql, events, chunk=1):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    for s in range(0, len(events), chunk):
        part = events[s:s + chunk]
        o.send_many("S", part, batch=chunk > 1)
        g.send_many("S", part, batch=chunk > 1)
    return o, g


@pytest.mark.parametrize("chunk", [1, 7])
def test_pattern_with_nulls_on_nfa(chunk, monkeypatch):
    monkeypatch.setenv("SG_PATHS", "nfa")
    ql = (S + " @info(name='query1') from every e1=S[price > 20] -> "
          "e2=S[volume > e1.volume or symbol == e1.symbol] "
          "select e1.symbol, e2.price, e2.volume, e2.price + e1.price as tot insert into Out;")
    o, g = _both(ql, _events(600, 1), chunk)
    assert g.path("query1") == "nfa"
    go, oo = g.outputs(), o.outputs()
    assert len(oo) > 0
    assert go == oo


def test_partitioned_pattern_with_nulls():
    ql = (S + " partition with (symbol of S) begin @info(name='query1') from every e1=S[price > 30] -> "
          "e2=S[price > e1.price] -> e3=S[volume < e2.volume] "
          "select e1.symbol, e1.price as p1, e3.volume as v3 insert into Out; end;")
    evs = [(t, [d[0] if d[0] is not None else "A", d[1], d[2]]) for t, d in _events(800, 2)]
    o, g = _both(ql, evs)
    assert g.path("query1") == "nfa"
    assert g.outputs() == o.outputs()


@pytest.mark.parametrize("chunk", [1, 5])
def test_window_aggregators_with_nulls(chunk):
    ql = (S + " @info(name='query1') from S[price > 10 or volume > 500]#window.length(4) "
          "select symbol, sum(volume) as v, avg(price) as a, max(price) as m, count() as c "
          "group by symbol insert all events into Out;")
    o, g = _both(ql, _events(700, 3), chunk)
    assert g.path("query1") == "window"
    go, oo = g.outputs(), o.outputs()
    assert len(oo) > 0
    assert go == oo


def test_scan_path_refuses_nulls():
    ql = (S + " @info(name='query1') from every e1=S[price > 20] -> e2=S[price > e1.price] within 1 sec "
          "select e1.symbol, e2.price insert into Out;")
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "followed_by"
    g.send_many("S", [(1, ["A", 30.0, 1])], batch=False)
    with pytest.raises(SiddhiGfxError) as e:
        g.send_many("S", [(2, ["A", None, 1])], batch=False)
    assert e.value.code == -2
