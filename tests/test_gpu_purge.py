"""@purge on partitions (PartitionRuntimeImpl.java:120-147, 346-402) on the device
paths, against the oracle on the same streams: bit-exact rows, timestamps and callback grouping.

Streams are bursty per key (keys fall idle for longer than idle.period and come back), so instances are
cleaned and re-initialised many times: window contents and aggregators start over (general window
path), partial matches and count chains are dropped (NFA lanes), time-window Scheduler states of cleaned
keys never fire.  The keyed scan path keeps a purge only where it is invisible (playback, idle.period >=
within); otherwise the query runs on the NFA path.
"""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

S = synth.STOCK_STREAM
TYPES = ["STRING", "FLOAT", "INT"]


def _bursty(n, seed, k):
    """Keys in bursts: each event keeps the previous key with p = 0.7, else a Zipf-ish draw; gaps of
    0..400 ms, so a key's next burst is often seconds away."""
    rng = np.random.default_rng(seed)
    d = synth.stock_ticks(n, seed=seed, k=k)
    w = 1.0 / np.arange(1, k + 1)
    w /= w.sum()
    sym = np.empty(n, np.int32)
    cur = 0
    for i in range(n):
        if rng.random() > 0.7:
            cur = int(rng.choice(k, p=w))
        sym[i] = cur
    d["symbol"] = sym
    d["ts"] = synth.T0 + np.cumsum(rng.integers(0, 400, n)).astype(np.int64)
    return d


def _run(ql, n, k, path, seed=5, chunk=None, clock=False):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == path, (g.path("query1"), ql)
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    d = _bursty(n, seed, k)
    cols = [gi[d["symbol"]], d["price"], d["volume"]]
    raw = raw_matrix(TYPES, cols)
    si = o.L.or_stream_index(o.h, b"StockStream")
    step = chunk or 1
    rng = np.random.default_rng(seed + 1)
    for s in range(0, n, step):
        if clock and rng.random() < 0.1:   # clock advances between sends (fire time-window timers)
            t = int(d["ts"][s]) - 1 - int(rng.integers(0, 300))
            if t > 0:
                o.set_time(t)
                g.set_time(t)
        o.send_columns(si, d["ts"][s:s + step], raw[s:s + step], None, chunk is not None)
        g.send_columns("StockStream", d["ts"][s:s + step], [c[s:s + step] for c in cols], chunk is not None)
    out = g.raw_outputs()
    compare_raw(o.raw_outputs(), out, 4)
    return int(np.sum(out[0]["n_in"])) + int(np.sum(out[0]["n_rm"]))


PURGE = "@purge(enable='true', interval='1 sec', idle.period='2 sec') "


def _part(body, purge=PURGE, playback=False):
    return (("@app:playback " if playback else "") + S + " " + purge +
            "partition with (symbol of StockStream) begin @info(name='query1') " + body + " end;")


CASES = {
    "window_length_avg": ("from StockStream#window.length(3) select symbol, avg(price) as ap, count() as c "
                          "insert into Out;", "window", None, False),
    "window_batch_all": ("from StockStream#window.lengthBatch(3) select symbol, sum(volume) as v "
                         "insert all events into Out;", "window", 4, False),
    "window_time_timers": ("from StockStream#window.time(3 sec) select symbol, sum(volume) as v, count() as c "
                           "insert all events into Out;", "window", None, True),
    "nfa_every_no_within": ("from every e1=StockStream[price > 30] -> e2=StockStream[price > e1.price] "
                            "select e1.symbol, e1.price as p1, e2.price as p2 insert into Out;", "nfa", None, False),
    "nfa_count": ("from every e1=StockStream -> e2=StockStream[price > e1.price]<2:4> -> "
                  "e3=StockStream[price < e2[last].price] select e1.symbol, e1.price as p1, e3.price as p3 "
                  "insert into Out;", "nfa", None, False),
    "nfa_aggregator": ("from every e1=StockStream[price > 50] -> e2=StockStream[price < e1.price] "
                       "select e1.symbol, sum(e2.volume) as tv, count() as c insert into Out;", "nfa", None, False),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_purge_parity(name):
    body, path, chunk, clock = CASES[name]
    assert _run(_part(body), 6000, 12, path, chunk=chunk, clock=clock) > 0


def test_purge_changes_results():
    """The purge is observable on these streams (else the parity above proves little)."""
    body = CASES["window_length_avg"][0]
    ql_on, ql_off = _part(body), _part(body, purge="")
    d = _bursty(3000, 5, 12)
    outs = []
    for ql in (ql_on, ql_off):
        o = OracleApp(ql); o.add_query_callback("query1"); o.start()
        ids = intern_symbols(o, 12)
        raw = raw_matrix(TYPES, [ids[d["symbol"]], d["price"], d["volume"]])
        o.send_columns(o.L.or_stream_index(o.h, b"StockStream"), d["ts"], raw, None, False)
        outs.append(o.outputs())
    assert outs[0] != outs[1]


KEYED = ("from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 1 sec "
         "select e1.symbol, e2.price insert into Out;")


def test_keyed_path_keeps_an_invisible_purge():
    # playback and idle.period (2 s) >= within (1 s): nothing a purge cleans could still match
    assert _run(_part(KEYED, playback=True), 8000, 12, "keyed_followed_by") > 0


@pytest.mark.parametrize("purge,playback", [("@purge(enable='true', interval='1 sec', idle.period='0 sec') ", True),
                                            (PURGE, False)])
def test_keyed_shape_with_a_visible_purge_runs_on_the_nfa(purge, playback):
    assert _run(_part(KEYED, purge=purge, playback=playback), 6000, 12, "nfa") > 0


def test_purge_disabled_is_ignored():
    ql = _part(KEYED, purge="@purge(enable='false', idle.period='1 sec') ")
    assert _run(ql, 4000, 12, "keyed_followed_by") > 0


def test_purge_with_absent_states_is_refused_per_query():
    ql = _part("from every e1=StockStream -> not StockStream[price > 90] for 1 sec select e1.symbol "
               "insert into Out;")
    g = GpuApp(ql, allow_partial=True)
    assert g.path("query1") == "unsupported"


@pytest.mark.parametrize("name", ["window_length_avg", "nfa_every_no_within"])
def test_purge_snapshot_round_trip(name):
    body, path, _chunk, _clock = CASES[name]
    ql = _part(body)
    n, k, cut = 4000, 12, 1700
    d = _bursty(n, 9, k)

    def new():
        g = GpuApp(ql); g.add_query_callback("query1"); g.start()
        return g, intern_symbols(g, k)

    def send(g, ids, lo, hi):
        g.send_columns("StockStream", d["ts"][lo:hi], [ids[d["symbol"][lo:hi]], d["price"][lo:hi],
                                                       d["volume"][lo:hi]], False)

    a, ids = new()
    assert a.path("query1") == path
    for i in range(n):
        send(a, ids, i, i + 1)
    want = a.outputs()
    b, _ = new()
    for i in range(cut):
        send(b, ids, i, i + 1)
    state = b.snapshot()
    got = b.outputs()
    c, _ = new()
    c.restore(state)
    for i in range(cut, n):
        send(c, ids, i, i + 1)
    got += c.outputs()
    assert len(want) > 0 and got == want
