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


def _oracle_outputs(ql, k, d, cuts, chunk):
    """The oracle (one runtime) fed the same sends: the reference's answer for the whole stream."""
    from oracle.pyoracle import OracleApp
    from synth_run import raw_matrix
    o = OracleApp(ql)
    o.add_query_callback("query1")
    o.start()
    ids = intern_symbols(o, k)
    si = o.L.or_stream_index(o.h, b"StockStream")
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [ids[d["symbol"]], d["price"], d["volume"]])
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        for s in range(lo, hi, chunk):
            e = min(hi, s + chunk)
            o.send_columns(si, d["ts"][s:e], raw[s:e], None, chunk > 1)
    return o.outputs()


def _round_trip(ql, n, k, cut, chunk=1, seed=3, rr=False):
    d = synth.stock_ticks_rr(n, seed, k) if rr else synth.stock_ticks(n, seed=seed, k=k, e=1)
    want = _oracle_outputs(ql, k, d, [0, cut, n], chunk)
    a, ids = _new(ql, k)
    _send(a, ids, d, 0, n, chunk)
    assert a.outputs() == want                       # one device run equals the oracle
    b, _ = _new(ql, k)
    _send(b, ids, d, 0, cut, chunk)
    state = b.snapshot()
    got = b.outputs()
    c, _ = _new(ql, k)
    c.restore(state)
    _send(c, ids, d, cut, n, chunk)
    got += c.outputs()
    assert len(want) > 0
    assert got == want                               # B + C (through the snapshot) equals the oracle
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


@pytest.mark.parametrize("name", ["count_sequence", "partitioned_absent", "window_expired"])
def test_failed_restore_leaves_a_restarted_runtime(name):
    """A snapshot whose query state is cut short fails to load and leaves the app as sg_reset does (clock,
    @purge schedules, start-time state of a started app): the whole stream then gives the oracle's answer."""
    ql, n, k, chunk = CASES[name]
    n = n // 2 // chunk * chunk
    d = synth.stock_ticks_rr(n, 3, k) if name == "partitioned_absent" else synth.stock_ticks(n, seed=3, k=k, e=1)
    b, ids = _new(ql, k)
    _send(b, ids, d, 0, n // 2 // chunk * chunk, chunk)
    state = b.snapshot()
    c, _ = _new(ql, k)
    _send(c, ids, d, 0, n // 4 // chunk * chunk, chunk)   # some state of its own before the failed restore
    c.outputs()
    with pytest.raises(SiddhiGfxError):
        c.restore(state[:-9])
    _send(c, ids, d, 0, n, chunk)
    assert c.outputs() == _oracle_outputs(ql, k, d, [0, n], chunk)


# The scan paths (SURVEY §8 A1/A9 followed-by, A13-A15 window + aggregation): run B takes the first part
# (several flushes), is snapshotted, and C restores it and takes the rest.  B + C is compared with the
# ORACLE over the whole stream (not with another device run), with the raw row/timestamp/grouping bar.
SCAN_CASES = {
    # unkeyed `every e1 -> e2 within 1 sec` (config 1): pending starts carried through the snapshot
    "followed_by": (synth.CONFIG1_QL, "followed_by", 60_000, 200, 1, 2),
    # keyed `partition with ... every e1 -> e2 within 1 sec` (config 4, the headline path): carried starts
    "keyed_followed_by": (synth.CONFIG4_QL, "keyed_followed_by", 200_000, 20_000, 40, 2),
    # filter + length(1000) + group-by sum/avg/count (config 2): window contents and group states
    "window_agg": (synth.CONFIG2_QL, "window_agg", 50_000, 100, 1, 4),
}


@pytest.mark.parametrize("name", sorted(SCAN_CASES))
@pytest.mark.parametrize("frac", [0.37, 0.8])
def test_scan_path_snapshot_matches_oracle(name, frac):
    from oracle.pyoracle import OracleApp
    from synth_run import compare_raw, raw_matrix
    ql, path, n, k, e, ncols = SCAN_CASES[name]
    d = synth.stock_ticks(n, seed=synth.SEEDS[4] + 3, k=k, e=e)
    cut = int(n * frac)
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    oi = intern_symbols(o, k)
    b, gi = _new(ql, k)
    assert b.path("query1") == path
    assert np.array_equal(oi, gi)
    cols = [gi[d["symbol"]], d["price"], d["volume"]]
    types = ["STRING", "FLOAT", "INT"]
    part = lambda lo, hi: (d["ts"][lo:hi], [c[lo:hi] for c in cols])   # noqa: E731
    # B: the first part in two flushes (the second carries the first's open state), then the snapshot
    half = cut // 2
    b.send_columns("StockStream", *part(0, half), True)
    parts = [b.raw_outputs()]
    b.send_columns("StockStream", *part(half, cut), True)
    state = b.snapshot()
    parts.append(b.raw_outputs())
    assert b.buffered("query1") < cut                    # compacted: the snapshot holds open state only
    c, _ = _new(ql, k)
    c.restore(state)
    c.send_columns("StockStream", *part(cut, n), True)
    parts.append(c.raw_outputs())
    si = o.L.or_stream_index(o.h, b"StockStream")
    raw = raw_matrix(types, cols)
    for lo, hi in ((0, half), (half, cut), (cut, n)):      # the same send chunks as B + C
        o.send_columns(si, d["ts"][lo:hi], raw[lo:hi], None, True)
    cb = {f: np.concatenate([p[0][f] for p in parts]) for f in parts[0][0]}
    merged = (cb, np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]),
              np.concatenate([p[3] for p in parts]))
    compare_raw(o.raw_outputs(), merged, ncols)
    assert len(merged[1]) > 0


def test_scan_snapshot_after_device_ingest_is_refused():
    import torch
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    g, ids = _new(synth.CONFIG4_QL, 10)
    d = synth.stock_ticks(1000, seed=1, k=10)
    ts = torch.from_numpy(d["ts"]).to(dev)
    sy = torch.from_numpy(ids[d["symbol"]].astype(np.int32)).to(dev)
    pr = torch.from_numpy(d["price"]).to(dev)
    torch.cuda.synchronize()
    g.push_device("StockStream", 1000, ts.data_ptr(), [sy.data_ptr(), pr.data_ptr(), 0])
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
