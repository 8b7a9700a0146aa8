"""Absent states (`not S[f] for T`, AbsentStreamPreStateProcessor / Scheduler) on the device NFA
lanes, against the oracle, on seeded two-stream streams in playback mode.  The reference's own absent KATs
(tests/golden/kats.json, absent/*TestCase.java) run through test_gpu_parity.py."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, raw_matrix

pytestmark = pytest.mark.gpu

STREAMS = ("@app:playback define stream A (sym string, price float, vol int); "
           "define stream B (sym string, price float, vol int); ")


def _streams(n, seed, gap):
    r = synth.splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(seed))
    which = (r & np.uint64(3)).astype(np.int64)            # 3/4 A, 1/4 B
    price = ((r >> np.uint64(8)) % np.uint64(9000)).astype(np.float32) / np.float32(100.0) + np.float32(10.0)
    vol = ((r >> np.uint64(30)) % np.uint64(1000)).astype(np.int32)
    ts = 1_000 + np.cumsum(((r >> np.uint64(40)) % np.uint64(gap)).astype(np.int64))
    return which, price, vol, ts


def _run(ql, n, seed, gap, ncols, batch_every=None, sleeps=False):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    sid_o, sid_g = o.intern("S0"), g.intern("S0")
    assert sid_o == sid_g
    which, price, vol, ts = _streams(n, seed, gap)
    sa, sb = o.L.or_stream_index(o.h, b"A"), o.L.or_stream_index(o.h, b"B")
    for i in range(n):
        name, si = ("B", sb) if which[i] == 0 else ("A", sa)
        cols = [np.array([sid_o], np.int32), price[i:i + 1], vol[i:i + 1]]
        raw = raw_matrix(["STRING", "FLOAT", "INT"], cols)
        o.send_columns(si, ts[i:i + 1], raw, None, False)
        g.send_columns(name, ts[i:i + 1], cols, False)
        if sleeps and i % 97 == 96:
            o.sleep(0); g.sleep(0)
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    return g


@pytest.mark.parametrize("gap", [7, 40])
def test_followed_by_absent(gap):
    ql = STREAMS + ("@info(name='query1') from e1=A[price > 50] -> not B[price > e1.price] for 60 milliseconds "
                    "select e1.price as p, e1.vol as v insert into Out;")
    _run(ql, 3_000, 41, gap, 2)


def test_every_followed_by_absent():
    ql = STREAMS + ("@info(name='query1') from every e1=A[price > 60] -> not B[price > e1.price] for 30 milliseconds "
                    "select e1.price as p insert into Out;")
    _run(ql, 4_000, 42, 12, 1)


def test_absent_start_then_stream():
    ql = STREAMS + ("@info(name='query1') from not B[price > 90] for 45 milliseconds -> e2=A[price > 70] "
                    "select e2.price as p, e2.vol as v insert into Out;")
    _run(ql, 3_000, 43, 9, 2)


def test_every_absent_start():
    ql = STREAMS + ("@info(name='query1') from every not B[price > 80] for 25 milliseconds -> e2=A "
                    "select e2.price as p insert into Out;")
    _run(ql, 2_000, 44, 6, 1)


def test_absent_within_sequence():
    ql = STREAMS + ("@info(name='query1') from every e1=A[price > 40], not B for 20 milliseconds "
                    "select e1.price as p insert into Out;")
    _run(ql, 2_500, 45, 60, 1)
