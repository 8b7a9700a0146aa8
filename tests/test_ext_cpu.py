"""The window / aggregator extension ABI (include/siddhi_gfx_ext.h) against the oracle.

The extension classes replace `length`, `time`, `lengthBatch` and `sum/avg/count/min/max` one by one, so
the test drives them the way the stock runtime would: every send is one processEventChunk call of the
window (playback: the Scheduler's TIMER chunks fire first, InputHandler.java:59-70), each output chunk
goes through the selector (no group-by: the chunk's last event carries the aggregates, QuerySelector
.processInBatchNoGroupBy :271-313), and the result must equal the oracle's QueryCallback for the same
query: the events (by id), their types, timestamps and aggregate values, chunk by chunk.  Host code: no
GPU needed."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "siddhi_amd", "_build", "libsiddhi_gfx.so")
WIN = {"length": 1, "time": 2, "lengthBatch": 3}
AGG = {"sum": 0, "avg": 1, "count": 2, "min": 3, "max": 4}
T_INT, T_FLOAT = 1, 3
S = "define stream S (id int, price float, volume int);"


@pytest.fixture(scope="module")
def L():
    return load_lib()


def load_lib():
    L = C.CDLL(LIB)
    P, I64 = C.c_void_p, C.c_int64
    L.sg_window_create.argtypes = [C.c_int, I64, C.c_int, C.c_int, C.POINTER(P)]
    L.sg_window_destroy.argtypes = [P]
    L.sg_window_process.argtypes = [P, I64, P, P, I64]
    L.sg_window_on_time.argtypes = [P, I64]
    L.sg_window_next_deadline.argtypes = [P]
    L.sg_window_next_deadline.restype = I64
    L.sg_window_out_sizes.argtypes = [P, C.POINTER(I64), C.POINTER(I64)]
    L.sg_window_out_copy.argtypes = [P, P, P, P, P]
    L.sg_window_snapshot.argtypes = [P, C.POINTER(P), C.POINTER(I64)]
    L.sg_window_restore.argtypes = [P, P, I64]
    L.sg_free_buffer.argtypes = [P]
    L.sg_agg_create.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(P)]
    L.sg_agg_destroy.argtypes = [P]
    L.sg_agg_process.argtypes = [P, I64, P, P, P, P, P]
    L.sg_agg_can_destroy.argtypes = [P]
    L.sg_agg_out_type.argtypes = [P]
    L.sg_last_error.restype = C.c_char_p
    return L


class Window:
    def __init__(self, L, kind, param, stream_current=False, expired_on=True):
        self.L = L
        self.h = C.c_void_p()
        assert L.sg_window_create(WIN[kind], param, int(stream_current), int(expired_on), C.byref(self.h)) == 0

    def process(self, ids, ts, now):
        ids = np.ascontiguousarray(ids, np.int64)
        ts = np.ascontiguousarray(ts, np.int64)
        assert self.L.sg_window_process(self.h, len(ids), ids.ctypes.data, ts.ctypes.data, now) == 0

    def on_time(self, now):
        assert self.L.sg_window_on_time(self.h, now) == 0

    def chunks(self):
        n, c = C.c_int64(), C.c_int64()
        self.L.sg_window_out_sizes(self.h, C.byref(n), C.byref(c))
        ids = np.empty(n.value, np.int64); ty = np.empty(n.value, np.int32); ts = np.empty(n.value, np.int64)
        end = np.empty(c.value, np.int64)
        assert self.L.sg_window_out_copy(self.h, ids.ctypes.data, ty.ctypes.data, ts.ctypes.data, end.ctypes.data) == 0
        out, b = [], 0
        for e in end:
            out.append((ids[b:e], ty[b:e], ts[b:e]))
            b = e
        return out


class Agg:
    def __init__(self, L, kind, in_type, track):
        self.L = L
        self.h = C.c_void_p()
        assert L.sg_agg_create(AGG[kind], in_type, int(track), C.byref(self.h)) == 0

    def process(self, types, vals):
        n = len(types)
        types = np.ascontiguousarray(types, np.int32)
        vals = np.ascontiguousarray(vals, np.int64)
        out = np.empty(n, np.int64); nul = np.empty(n, np.uint8)
        assert self.L.sg_agg_process(self.h, n, types.ctypes.data, vals.ctypes.data, None, out.ctypes.data,
                                     nul.ctypes.data) == 0
        return out, nul


def _stream(n, seed):
    d = synth.stock_ticks(n, seed=seed, k=10)
    rng = np.random.default_rng(seed)
    d["ts"] = synth.T0 + np.cumsum(rng.integers(0, 900, n)).astype(np.int64)
    return d


def _oracle(ql, d):
    o = OracleApp("@app:playback " + S + " @info(name='q') " + ql)
    o.add_query_callback("q")
    o.start()
    for i in range(len(d["ts"])):
        o.send("S", [i, float(d["price"][i]), int(d["volume"][i])], ts=int(d["ts"][i]))
    cbs, ts, raw, nul = o.raw_outputs()
    out, r = [], 0
    for c in range(len(cbs["kind"])):
        k = int(cbs["n_in"][c]) + int(cbs["n_rm"][c])
        out.append((raw[r:r + k], nul[r:r + k], ts[r:r + k], int(cbs["n_in"][c])))
        r += k
    return out


WINDOWS = [("length", 4, False), ("length", 0, False), ("time", 2000, False), ("lengthBatch", 3, False),
           ("lengthBatch", 3, True), ("lengthBatch", 0, False)]


def _drive(L, kind, param, sc, d, aggs=()):
    """The stock runtime around the extension window (and aggregators): -> one entry per QueryCallback."""
    w = Window(L, kind, param, sc, expired_on=True)
    # min/max trackFutureStates: a sliding window or expired output (`all events` here)
    ag = [(Agg(L, a, t, True), col) for a, t, col in aggs]
    got = []
    for i in range(len(d["ts"])):
        t = int(d["ts"][i])
        w.on_time(t)                        # playback: due timers before the event is dispatched
        w.process([i], [t], t)
        for ids, ty, ts in w.chunks():
            keep = ty != 3                  # RESET reaches the aggregators, never the output
            if not aggs:
                cur, exp = ids[keep & (ty == 0)], ids[keep & (ty == 1)]
                got.append((list(cur) + list(exp), list(ts[keep & (ty == 0)]) + list(ts[keep & (ty == 1)]),
                            len(cur)))
                continue
            res = []
            for a, col in ag:
                vals = np.array([d[col][j].view(np.uint32) if col == "price" else d[col][j] for j in ids], np.int64)
                res.append(a.process(ty, vals))
            last = np.nonzero(keep)[0]
            if len(last):
                j = last[-1]
                got.append(([(r[0][j], r[1][j]) for r in res], int(ts[j]), int(ty[j] == 0)))
    return got


@pytest.mark.parametrize("kind,param,sc", WINDOWS)
def test_window_extension_matches_the_query(L, kind, param, sc):
    d = _stream(400, 7)
    args = f"{param // 1000} sec" if kind == "time" else f"{param}, true" if sc else f"{param}"
    want = _oracle(f"from S#window.{kind}({args}) select id insert all events into Out;", d)
    got = _drive(L, kind, param, sc, d)
    assert len(got) == len(want) and len(got) > 0
    for (ids, ts, ncur), (raw, nul, ots, nin) in zip(got, want):
        assert ids == list(raw[:, 0]) and ts == list(ots) and ncur == nin


@pytest.mark.parametrize("kind,param", [("length", 5), ("time", 3000), ("lengthBatch", 4)])
def test_aggregator_extensions_match_the_selector(L, kind, param):
    d = _stream(500, 11)
    args = f"{param // 1000} sec" if kind == "time" else f"{param}"
    want = _oracle(f"from S#window.{kind}({args}) select sum(price) as s, avg(price) as a, count() as c, "
                   f"min(volume) as mn, max(price) as mx, sum(volume) as sv insert all events into Out;", d)
    aggs = [("sum", T_FLOAT, "price"), ("avg", T_FLOAT, "price"), ("count", T_INT, "volume"),
            ("min", T_INT, "volume"), ("max", T_FLOAT, "price"), ("sum", T_INT, "volume")]
    got = _drive(L, kind, param, False, d, aggs)
    assert len(got) == len(want) and len(got) > 0
    for (vals, ts, cur), (raw, nul, ots, nin) in zip(got, want):
        assert ts == int(ots[-1]) and cur == int(nin == 1)
        for k, (v, isnull) in enumerate(vals):
            assert bool(isnull) == bool(nul[0, k])
            if not isnull:
                assert v == raw[0, k], (k, v, raw[0, k])


def test_min_max_deque_value_removal_quirk(L):
    # MinAttributeAggregatorExecutor.java:175-203: an expiry removes the FIRST deque entry equal to its value.
    # Adds 3a, 2, 3b keep the deque [2, 3b]; expiring 3a removes 3b, expiring 2 empties it: min is null
    # while 3b is still in the window -- the reference's answer, kept
    a = Agg(L, "min", T_INT, True)
    out, nul = a.process([0, 0, 0, 1, 1], [3, 2, 3, 3, 2])
    assert list(out[:4]) == [3, 2, 2, 2] and list(nul) == [0, 0, 0, 0, 1]
    assert L.sg_agg_can_destroy(a.h) == 1


def test_long_sum_removes_through_double(L):
    # SumAttributeAggregatorExecutor.processRemove(double): sum = (long) (sum - (double) x)
    a = Agg(L, "sum", 2, False)   # LONG
    big = (1 << 60) + 1
    out, nul = a.process([0, 0, 1], [big, 3, 3])
    assert out[1] == big + 3 and out[2] == int(float(big + 3) - 3.0)


def test_window_snapshot_round_trip(L):
    d = _stream(300, 3)
    a, b = Window(L, "time", 2000), Window(L, "time", 2000)
    for i in range(300):
        t = int(d["ts"][i])
        if i == 150:
            buf, n = C.c_void_p(), C.c_int64()
            assert L.sg_window_snapshot(b.h, C.byref(buf), C.byref(n)) == 0
            c = Window(L, "time", 2000)
            assert L.sg_window_restore(c.h, buf, n) == 0
            L.sg_free_buffer(buf)
            b = c
        for w in (a, b):
            w.on_time(t)
            w.process([i], [t], t)
        ca, cb = a.chunks(), b.chunks()
        assert len(ca) == len(cb) and all((x[0] == y[0]).all() and (x[1] == y[1]).all() for x, y in zip(ca, cb))
    assert L.sg_window_next_deadline(a.h) == L.sg_window_next_deadline(b.h) != -(1 << 63)


def test_bad_arguments_are_refused(L):
    h = C.c_void_p()
    assert L.sg_window_create(9, 3, 0, 0, C.byref(h)) == -1
    assert L.sg_window_create(1, 3, 1, 0, C.byref(h)) == -1     # streamCurrentEvents on length
    assert L.sg_agg_create(0, 0, 0, C.byref(h)) == -1           # sum of a STRING
    assert b"INT, LONG, FLOAT or DOUBLE" in L.sg_last_error()


def test_time_window_scheduler_gets_every_deadline(L):
    """The Java Time extension forwards the deadlines sg_window_take_deadlines hands out to its Scheduler
    (TimeWindowProcessor.java:158-160: one notifyAt(ts + T) per new timestamp); the Scheduler alone then
    decides when TIMER chunks run.  Two events at distinct timestamps, then only clock advances: both
    deadlines must fire, as the query (non-playback, sleep-driven) expires both events."""
    L.sg_window_take_deadlines.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int64]
    L.sg_window_take_deadlines.restype = C.c_int64
    w = Window(L, "time", 5000)
    sched = []                                   # the Scheduler's toNotifyQueue

    def take():
        n = L.sg_window_take_deadlines(w.h, None, 0)
        buf = (C.c_int64 * max(n, 1))()
        assert L.sg_window_take_deadlines(w.h, buf, n) == n
        sched.extend(buf[:n])

    got = []
    for now, ev in [(1000, 0), (2000, 1), (2000, 2), (6500, None), (7500, None)]:
        while sched and sched[0] <= now:         # sendTimerEvents: one TIMER chunk per due deadline
            sched.pop(0)
            w.on_time(now)
        if ev is not None:
            w.process([ev], [now], now)
            take()
        for ids, ty, ts in w.chunks():
            got.append([(int(i), int(t), int(s)) for i, t, s in zip(ids, ty, ts)])
    assert L.sg_window_take_deadlines(w.h, None, 0) == 0
    expired = [c for c in got if c and c[0][1] == 1]
    assert expired == [[(0, 1, 6500)], [(1, 1, 7500), (2, 1, 7500)]]
    o = OracleApp(S + " @info(name='q') from S#window.time(5 sec) select id insert all events into Out;")
    o.add_query_callback("q")
    o.start()
    for now, ev in [(1000, 0), (2000, 1), (2000, 2), (6500, None), (7500, None)]:
        o.set_time(now)
        if ev is not None:
            o.send("S", [ev, 1.0, 1])
    cbs, ts, raw, nul = o.raw_outputs()
    rm = [(int(raw[r, 0]), int(ts[r])) for c, r0 in enumerate(np.cumsum(np.r_[0, cbs["n_in"] + cbs["n_rm"]])[:-1])
          for r in range(r0 + int(cbs["n_in"][c]), r0 + int(cbs["n_in"][c] + cbs["n_rm"][c]))]
    assert rm == [(0, 6500), (1, 7500), (2, 7500)]


def test_aggregator_snapshot_round_trip(L):
    L.sg_agg_snapshot.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    L.sg_agg_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    rng = np.random.default_rng(5)
    ty = rng.choice([0, 0, 1], 200).astype(np.int32)
    vals = rng.integers(-50, 50, 200)
    for kind in AGG:
        a, b = Agg(L, kind, T_INT, True), Agg(L, kind, T_INT, True)
        a.process(ty[:120], vals[:120])
        b.process(ty[:120], vals[:120])
        buf, n = C.c_void_p(), C.c_int64()
        assert L.sg_agg_snapshot(b.h, C.byref(buf), C.byref(n)) == 0
        c = Agg(L, kind, T_INT, True)
        assert L.sg_agg_restore(c.h, buf, n) == 0
        other = Agg(L, "sum" if kind != "sum" else "avg", T_INT, True)
        assert L.sg_agg_restore(other.h, buf, n) == -1           # another aggregator's state is refused
        L.sg_free_buffer(buf)
        oa, na = a.process(ty[120:], vals[120:])
        oc, nc = c.process(ty[120:], vals[120:])
        assert (oa == oc).all() and (na == nc).all(), kind
