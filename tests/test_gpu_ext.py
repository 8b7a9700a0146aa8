"""The window / aggregator extension ABI on its device path (ext.hip: k_ext_len, k_ext_time_*, k_ext_batch_*,
k_ext_agg_check / _delta / _out with a hipcub segmented scan, k_ext_minmax) against the oracle's QueryCallbacks
(AbstractStreamProcessor.java:66-98, AttributeAggregatorExecutor.execute :59-67).

The stock runtime around the extension classes is driven with batch sends of 5,000 events (one
processEventChunk per `InputHandler.send(Event[])`, the chunk's clock its last timestamp in playback), so every
chunk is past SG_EXT_DEVICE_MIN and runs on the device: the length window's output chunk (EXPIRED before each
CURRENT once full, the expired ones re-stamped with the chunk's clock) must equal the oracle's in / removed rows,
ids and timestamps; the aggregators over that chunk (count, sum and avg of an INT and of a FLOAT column: exact
integer and fixed-point scans) must give the selector's batch output (QuerySelector.processInBatchNoGroupBy
:271-313: the chunk's last event), values and nulls bit for bit."""
import ctypes as C

import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
import test_ext_cpu as cpu
from test_ext_cpu import AGG, LIB, S, T_FLOAT, T_INT, WIN

pytestmark = pytest.mark.gpu

B = 5_000


@pytest.fixture(scope="module")
def L():
    L = cpu.load_lib()                  # (every entry point typed: sg_window_on_time takes an int64 clock)
    L.sg_ext_device_chunks.restype = C.c_int64
    return L


def _stream(n, seed):
    d = synth.stock_ticks(n, seed=seed, k=10, e=3)
    return d


def _oracle(ql, d):
    """The query on the stock runtime restated (oracle), one send(Event[]) per B events: -> per callback
    (rows, nulls, row timestamps, number of in-events)."""
    o = OracleApp("@app:playback " + S + " @info(name='q') " + ql)
    o.add_query_callback("q")
    o.start()
    si = o.L.or_stream_index(o.h, b"S")
    n = len(d["ts"])
    raw = np.zeros((n, 3), np.int64)
    raw[:, 0] = np.arange(n)
    raw[:, 1] = d["price"].view(np.uint32).astype(np.int64)
    raw[:, 2] = d["volume"]
    for lo in range(0, n, B):
        o.send_columns(si, d["ts"][lo:lo + B], raw[lo:lo + B], None, True)
    cbs, ts, rw, nul = o.raw_outputs()
    out, r = [], 0
    for c in range(len(cbs["kind"])):
        k = int(cbs["n_in"][c]) + int(cbs["n_rm"][c])
        out.append((rw[r:r + k], nul[r:r + k], ts[r:r + k], int(cbs["n_in"][c])))
        r += k
    return out


def _window_chunks(L, param, d):
    h = C.c_void_p()
    assert L.sg_window_create(WIN["length"], param, 0, 1, C.byref(h)) == 0
    n = len(d["ts"])
    got = []
    for lo in range(0, n, B):
        ids = np.arange(lo, min(n, lo + B), dtype=np.int64)
        ts = np.ascontiguousarray(d["ts"][lo:lo + B], np.int64)
        assert L.sg_window_process(h, len(ids), ids.ctypes.data, ts.ctypes.data, int(ts[-1])) == 0
        m, c = C.c_int64(), C.c_int64()
        L.sg_window_out_sizes(h, C.byref(m), C.byref(c))
        oid = np.empty(m.value, np.int64); ot = np.empty(m.value, np.int32); ots = np.empty(m.value, np.int64)
        end = np.empty(c.value, np.int64)
        assert L.sg_window_out_copy(h, oid.ctypes.data, ot.ctypes.data, ots.ctypes.data, end.ctypes.data) == 0
        assert c.value == 1
        got.append((oid, ot, ots))
    return got


@pytest.mark.parametrize("param", [1000, 7_000])
def test_length_window_extension_on_device(L, param):
    d = _stream(40_000, 5)
    before = L.sg_ext_device_chunks()
    got = _window_chunks(L, param, d)
    assert L.sg_ext_device_chunks() - before == len(got)            # every chunk ran on the device
    want = _oracle(f"from S#window.length({param}) select id insert all events into Out;", d)
    assert len(got) == len(want)
    for (oid, ot, ots), (raw, _nul, wts, nin) in zip(got, want):
        cur, exp = ot == 0, ot == 1
        assert list(oid[cur]) + list(oid[exp]) == list(raw[:, 0])
        assert list(ots[cur]) + list(ots[exp]) == list(wts)
        assert int(cur.sum()) == nin


@pytest.mark.parametrize("param", [1000, 7_000])
def test_aggregator_extensions_on_device(L, param):
    d = _stream(40_000, 9)
    want = _oracle(f"from S#window.length({param}) select count() as c, sum(volume) as sv, avg(volume) as av, "
                   f"sum(price) as sp, avg(price) as ap insert all events into Out;", d)
    aggs = [("count", T_INT, "volume"), ("sum", T_INT, "volume"), ("avg", T_INT, "volume"),
            ("sum", T_FLOAT, "price"), ("avg", T_FLOAT, "price")]
    hs = []
    for kind, t, _col in aggs:
        h = C.c_void_p()
        assert L.sg_agg_create(AGG[kind], t, 1, C.byref(h)) == 0
        hs.append(h)
    vals = {"volume": d["volume"].astype(np.int64), "price": d["price"].view(np.uint32).astype(np.int64)}
    before = L.sg_ext_device_chunks()
    got = _window_chunks(L, param, d)
    for (oid, ot, ots), (raw, nul, wts, nin) in zip(got, want):
        ot = np.ascontiguousarray(ot, np.int32)
        j = len(ot) - 1                                                 # the chunk's last event (no RESET here)
        assert int(wts[-1]) == int(ots[j]) and len(raw) == 1
        for k, ((kind, t, col), h) in enumerate(zip(aggs, hs)):
            v = np.ascontiguousarray(vals[col][oid])
            out = np.empty(len(ot), np.int64)
            on = np.empty(len(ot), np.uint8)
            assert L.sg_agg_process(h, len(ot), ot.ctypes.data, v.ctypes.data, None, out.ctypes.data,
                                    on.ctypes.data) == 0
            assert bool(on[j]) == bool(nul[0, k]), (kind, col)
            if not on[j]:
                assert out[j] == raw[0, k], (kind, col, out[j], raw[0, k])
    # the window chunks and every aggregator batch ran on the device
    assert L.sg_ext_device_chunks() - before == len(got) * (1 + len(aggs))


# ---- every window and aggregator, every chunk forced to the device (SG_EXT_DEVICE=1) ----

@pytest.fixture
def forced(monkeypatch):
    monkeypatch.setenv("SG_EXT_DEVICE", "1")


@pytest.mark.parametrize("kind,param,sc", [("length", 4, False), ("time", 2000, False), ("lengthBatch", 3, False),
                                           ("lengthBatch", 3, True), ("lengthBatch", 1, True)])
def test_every_window_on_device_per_event(L, forced, kind, param, sc):
    """Per-event sends (one chunk per event, timers between them) through the device window kernels, against the
    query on the oracle: rows, timestamps and in / removed split of every callback."""
    d = cpu._stream(400, 7)
    args = f"{param // 1000} sec" if kind == "time" else f"{param}, true" if sc else f"{param}"
    want = cpu._oracle(f"from S#window.{kind}({args}) select id insert all events into Out;", d)
    before = L.sg_ext_device_chunks()
    got = cpu._drive(L, kind, param, sc, d)
    assert L.sg_ext_device_chunks() - before == len(d["ts"])        # every chunk ran on the device
    assert len(got) == len(want) and len(got) > 0
    for (ids, ts, ncur), (raw, nul, ots, nin) in zip(got, want):
        assert ids == list(raw[:, 0]) and ts == list(ots) and ncur == nin


@pytest.mark.parametrize("kind,param", [("length", 5), ("time", 3000), ("lengthBatch", 4)])
def test_every_aggregator_on_device(L, forced, kind, param):
    """sum / avg / count / min / max (trackFutureStates: the deque with value-equality removal) on the device for
    every window kind, against the selector's output on the oracle."""
    d = cpu._stream(500, 11)
    args = f"{param // 1000} sec" if kind == "time" else f"{param}"
    want = cpu._oracle(f"from S#window.{kind}({args}) select sum(price) as s, avg(price) as a, count() as c, "
                       f"min(volume) as mn, max(price) as mx, sum(volume) as sv insert all events into Out;", d)
    aggs = [("sum", T_FLOAT, "price"), ("avg", T_FLOAT, "price"), ("count", T_INT, "volume"),
            ("min", T_INT, "volume"), ("max", T_FLOAT, "price"), ("sum", T_INT, "volume")]
    before = L.sg_ext_device_chunks()
    got = cpu._drive(L, kind, param, False, d, aggs)
    assert L.sg_ext_device_chunks() - before >= len(d["ts"]) + len(aggs)    # windows and aggregator batches
    assert len(got) == len(want) and len(got) > 0
    for (vals, ts, cur), (raw, nul, ots, nin) in zip(got, want):
        assert ts == int(ots[-1]) and cur == int(nin == 1)
        for k, (v, isnull) in enumerate(vals):
            assert bool(isnull) == bool(nul[0, k])
            if not isnull:
                assert v == raw[0, k], (k, v, raw[0, k])


def test_min_max_quirk_on_device(L, forced):
    a = cpu.Agg(L, "min", T_INT, True)
    before = L.sg_ext_device_chunks()
    out, nul = a.process([0, 0, 0, 1, 1], [3, 2, 3, 3, 2])
    assert L.sg_ext_device_chunks() - before == 1
    assert list(out[:4]) == [3, 2, 2, 2] and list(nul) == [0, 0, 0, 0, 1]


@pytest.mark.parametrize("kind,param,sc", [("time", 3, False), ("lengthBatch", 2_000, False),
                                           ("lengthBatch", 1_500, True)])
def test_batched_windows_on_device(L, kind, param, sc):
    """send(Event[]) chunks of 5,000 events (past SG_EXT_DEVICE_MIN: the device by default): the time window with
    its timers fired before each chunk at the chunk's clock, lengthBatch in both modes."""
    d = _stream(40_000, 13)
    args = f"{param} sec" if kind == "time" else f"{param}, true" if sc else f"{param}"
    want = _oracle(f"from S#window.{kind}({args}) select id insert all events into Out;", d)
    w = cpu.Window(L, kind, param * 1000 if kind == "time" else param, sc, expired_on=True)
    before = L.sg_ext_device_chunks()
    got = []
    n = len(d["ts"])
    for lo in range(0, n, B):
        ids = np.arange(lo, min(n, lo + B), dtype=np.int64)
        ts = np.ascontiguousarray(d["ts"][lo:lo + B], np.int64)
        now = int(ts[-1])
        w.on_time(now)
        w.process(ids, ts, now)
        for oid, ty, ots in w.chunks():
            keep = ty != 3
            cur, exp = keep & (ty == 0), keep & (ty == 1)
            if cur.sum() + exp.sum() == 0:
                continue
            got.append((list(oid[cur]) + list(oid[exp]), list(ots[cur]) + list(ots[exp]), int(cur.sum())))
    assert L.sg_ext_device_chunks() - before == (n + B - 1) // B
    assert len(got) == len(want) and len(got) > 0
    for (ids, ts, ncur), (raw, nul, ots, nin) in zip(got, want):
        assert ids == list(raw[:, 0]) and ts == list(ots) and ncur == nin
