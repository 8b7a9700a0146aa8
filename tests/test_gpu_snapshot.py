"""sg_snapshot / sg_restore round trips through the C ABI (SiddhiAppRuntime.snapshot() / restore(byte[])).

For each app: run A takes the whole stream; run B takes the first part, is snapshotted, and a fresh app C
created from the same descriptor restores that state and takes the rest.  B's callbacks followed by C's
must equal A's exactly (rows, timestamps, grouping): partial matches, count chains, Scheduler queues of
absent states, partition instances, window queues and aggregator states all survive the round trip."""
import numpy as np
import pytest

from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp, SiddhiGfxError
from synth_run import intern_symbols

pytestmark = pytest.mark.gpu

S = synth.STOCK_STREAM


def _new(ql, k):
    g = GpuApp(ql)
    g.add_query_callback("query1")
    g.start()
    return g, intern_symbols(g, k)


def _send(g, ids, d, lo, hi, chunk):
    for s in range(lo, hi, chunk):
        e = min(hi, s + chunk)
        g.send_columns("StockStream", d["ts"][s:e], [ids[d["symbol"][s:e]], d["price"][s:e], d["volume"][s:e]],
                       chunk > 1)


def _round_trip(ql, n, k, cut, chunk=1, seed=3, rr=False):
    d = synth.stock_ticks_rr(n, seed, k) if rr else synth.stock_ticks(n, seed=seed, k=k, e=1)
    a, ids = _new(ql, k)
    _send(a, ids, d, 0, n, chunk)
    want = a.outputs()
    b, _ = _new(ql, k)
    _send(b, ids, d, 0, cut, chunk)
    state = b.snapshot()
    got = b.outputs()
    c, _ = _new(ql, k)
    c.restore(state)
    _send(c, ids, d, cut, n, chunk)
    got += c.outputs()
    assert len(want) > 0
    assert got == want
    return len(state)


CASES = {
    "count_sequence": (synth.CONFIG3_QL, 20_000, 50, 1),
    "logical_partitioned": (synth.CONFIG5_QL, 20_000, 100, 1),
    "partitioned_absent": ("@app:playback " + S + " partition with (symbol of StockStream) begin "
                           "@info(name='query1') from every e1=StockStream[price > 80] -> "
                           "not StockStream[volume > 990] for 3 sec select e1.symbol, e1.price insert into Out; end;",
                           30_000, 40, 1),
    "pattern_aggregators": (S + " @info(name='query1') from every e1=StockStream[price > 60] -> "
                            "e2=StockStream[price < e1.price] select e1.symbol, sum(e2.volume) as tv, count() as c "
                            "group by e1.symbol insert into Out;", 8_000, 8, 1),
    "window_expired": (S + " @info(name='query1') from StockStream#window.length(50) select symbol, "
                       "sum(volume) as v, max(price) as m group by symbol insert all events into Out;", 10_000, 10, 7),
    "partitioned_batch": (S + " partition with (symbol of StockStream) begin @info(name='query1') "
                          "from StockStream#window.lengthBatch(6) select symbol, avg(price) as a "
                          "insert all events into Out; end;", 10_000, 30, 5),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("frac", [0.3, 0.71])
def test_snapshot_restore_round_trip(name, frac):
    ql, n, k, chunk = CASES[name]
    cut = int(n * frac) // chunk * chunk
    _round_trip(ql, n, k, cut, chunk, rr=name == "partitioned_absent")


def test_snapshot_of_a_scan_path_is_refused():
    g, ids = _new(synth.CONFIG1_QL, 10)
    d = synth.stock_ticks(100, seed=1, k=10)
    _send(g, ids, d, 0, 100, 100)
    with pytest.raises(SiddhiGfxError) as e:
        g.snapshot()
    assert e.value.code == -2


def test_restore_rejects_another_app():
    g, ids = _new(synth.CONFIG3_QL, 10)
    state = g.snapshot()
    h, _ = _new(S + " @info(name='query1') from StockStream#window.length(5) select symbol, price "
                "insert all events into Out;", 10)
    with pytest.raises(SiddhiGfxError):
        h.restore(state)
    with pytest.raises(SiddhiGfxError):
        g.restore(state[:len(state) // 2])
