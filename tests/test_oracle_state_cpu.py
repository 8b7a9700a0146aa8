"""The restatement's StreamPreState export (or_query_state_json, the oracle side of tests/test_gpu_nfa_state.py) on
a hand-checked case: `every e1=S[price > 20] -> e2=S[price > e1.price]` after prices 30 and 25 holds the first start
in e2's pending list (StreamPreStateProcessor.java:450-469 PendingStateEventList) and the second in its
new-and-every list (a new partial becomes visible at the NEXT arrival, updateState :307-323), each with its e1 event
in slot 0 and nothing in slot 1; 40 then completes both and is itself the only new start."""
import numpy as np

from oracle.pyoracle import OracleApp, f32
from siddhi_amd import synth


def _f(x):
    return int(np.float32(x).view(np.uint32))


def test_pending_states_after_two_starts():
    ql = synth.STOCK_STREAM + " @info(name='query1') from every e1=StockStream[price > 20] -> " \
                              "e2=StockStream[price > e1.price] select e1.price as p1, e2.price as p2 insert into Out;"
    o = OracleApp(ql)
    o.add_query_callback("query1")
    o.start()
    s = o.intern("S")
    o.send("StockStream", ["S", 30.0, 1], ts=100)
    o.send("StockStream", ["S", 25.0, 2], ts=200)
    st = o.state_map("query1")
    assert len(st["instances"]) == 1 and st["instances"][0]["key"] is None
    procs = st["instances"][0]["processors"]
    assert len(procs) == 2
    e2 = procs[1]
    assert [se["slots"][0] for se in e2["pending"]] == [[[100, s, _f(30.0), 1]]]
    assert [se["slots"][0] for se in e2["new_and_every"]] == [[[200, s, _f(25.0), 2]]]
    assert all(se["slots"][1] == [] for se in e2["pending"] + e2["new_and_every"])
    assert procs[0]["initialized"] and [se["ts"] for se in procs[0]["new_and_every"]] == [200]   # every re-seed
    o.send("StockStream", ["S", 40.0, 3], ts=300)
    e2 = o.state_map("query1")["instances"][0]["processors"][1]
    assert e2["pending"] == [] and [se["ts"] for se in e2["new_and_every"]] == [300]   # 40 starts a partial
    assert f32(30.0) == 30.0
