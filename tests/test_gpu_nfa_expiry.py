"""`within` expiry on the NFA lanes (StreamPreStateProcessor.expireEvents :325-361, isExpired
:118-129) against the oracle, bit for bit, on lists long enough to span several 64-entry chunks.

The lanes evaluate expiry as a bit mask per chunk -- one __ballot of is_expired over the wavefront when a wave runs
one partition instance (wide mode, few instances), a per-thread mask when a wave runs 64 instances (narrow) -- and
compact the survivors to popc-rank positions (nfa_lane.hpp `expire_events`).  Each shape runs in both modes, with
the ahead-of-time interpreter and with the query's compiled kernel, flushing every few thousand events so that
lists carry across flushes:
  * pending lists of ~260 open starts whose prefix expires (a rare second condition keeps them open);
  * newAndEvery lists: one event completes many partials at once, and a 150 ms gap in a bursty stream expires
    part of them before the next event moves them to pending;
  * a count/Kleene sequence with `within` (BASELINE config 3 plus expiry);
  * many partition keys (narrow mode by lane count, two lanes per workgroup)."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]
S = synth.STOCK_STREAM
PART = S + " partition with (symbol of StockStream) begin "

# pending lists: every e1 opens a partial that e2 rarely completes (price above e1.price + 60), so ~260 stay open
# within 300 ms at one event per ms and their prefix expires event by event
LONG_PENDING = ("from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price + 60] -> "
                "e3=StockStream[price > e2.price] within 300 milliseconds "
                "select e1.price as p1, e2.price as p2, e3.price as p3 insert into Out;")
# newAndEvery lists: an e2 completes every open e1 below its price at once, all of them entering e3's newAndEvery
BURST_NEW = ("from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] -> "
             "e3=StockStream[price > e2.price + 50] within 200 milliseconds "
             "select e1.price as p1, e2.price as p2, e3.price as p3 insert into Out;")
SEQ_WITHIN = ("from every e1=StockStream, e2=StockStream[price > e1.price]+, e3=StockStream[price < e2[last].price] "
              "within 40 milliseconds "
              "select e1.symbol, e1.price as p1, e2[last].price as p2, e3.price as p3 insert into Out;")


def q(body, part):
    return (PART + "@info(name='query1') " + body + " end;") if part else (S + " @info(name='query1') " + body)


def bursty(n, seed, k, e=1, burst=100, gap=150):
    """Bursts of `burst` ms at e events per ms, then a `gap` ms pause (part of every list expires across it)."""
    d = synth.stock_ticks(n, seed=seed, k=k, e=e)
    i = np.arange(n, dtype=np.int64) // e
    d["ts"] = (synth.T0 + i + (i // burst) * gap).astype(np.int64)
    return d


def _run(ql, d, k, ncols, chunk, monkeypatch, wide, compiled):
    monkeypatch.setenv("SG_NFA_RTC", "1" if compiled else "0")
    monkeypatch.setenv("SG_NFA_WIDE", "1" if wide else "0")
    for v in ("SG_NFA_SPEC", "SG_NFA_TPB"):
        monkeypatch.delenv(v, raising=False)
    # lists of several hundred partials: pools above the defaults (64 StateEvents, 256 nodes, 48 list entries per
    # processor; an overflow is SG_E_CAPACITY, never a truncated list)
    monkeypatch.setenv("SG_NFA_SE_CAP", "640")
    monkeypatch.setenv("SG_NFA_ND_CAP", "2048")
    monkeypatch.setenv("SG_NFA_LIST_CAP", "640")
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    seen = []
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]],
              chunk=chunk, flush_each=True,
              after=lambda: seen.append((g.kernel_ms("nfa_wide"), g.kernel_ms("nfa_compiled"))))
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    ran = [x for x in seen if x[1] >= 0]
    assert ran, seen
    return ran, g


MODES = [(True, False), (True, True), (False, False), (False, True)]
IDS = ["wide-interp", "wide-compiled", "narrow-interp", "narrow-compiled"]


@pytest.mark.parametrize("wide,compiled", MODES, ids=IDS)
def test_long_pending_prefix_expiry(monkeypatch, wide, compiled):
    d = synth.stock_ticks(24_000, seed=synth.SEEDS[1] + 11, k=5, e=1)
    ran, g = _run(q(LONG_PENDING, False), d, 5, 3, 4_000, monkeypatch, wide, compiled)
    assert all(w == (1 if wide else 0) and c == (1 if compiled else 0) for w, c in ran), ran
    assert g.match_count("query1") >= 0


@pytest.mark.parametrize("wide,compiled", MODES, ids=IDS)
def test_new_and_every_expiry_across_gaps(monkeypatch, wide, compiled):
    d = bursty(30_000, synth.SEEDS[1] + 12, 5)
    ran, _ = _run(q(BURST_NEW, False), d, 5, 3, 5_000, monkeypatch, wide, compiled)
    assert all(w == (1 if wide else 0) for w, _c in ran), ran


@pytest.mark.parametrize("wide,compiled", MODES, ids=IDS)
def test_partitioned_few_keys_long_lists(monkeypatch, wide, compiled):
    """8 keys at one event per key per ms: eight instances, each with ~260-entry lists."""
    d = bursty(48_000, synth.SEEDS[4] + 13, 8, e=8, burst=400, gap=120)
    _run(q(LONG_PENDING, True), d, 8, 3, 12_000, monkeypatch, wide, compiled)


@pytest.mark.parametrize("wide,compiled", MODES, ids=IDS)
def test_sequence_count_states_within(monkeypatch, wide, compiled):
    d = bursty(40_000, synth.SEEDS[3] + 14, 50, e=4, burst=60, gap=30)
    _run(q(SEQ_WITHIN, True), d, 50, 4, 10_000, monkeypatch, wide, compiled)


def test_many_keys_narrow_by_lane_count(monkeypatch):
    """3,000 instances: two lanes per workgroup, so the launch is narrow whatever SG_NFA_WIDE says."""
    d = bursty(90_000, synth.SEEDS[4] + 15, 3000, e=30, burst=200, gap=100)
    ran, _ = _run(q(BURST_NEW, True), d, 3000, 3, 30_000, monkeypatch, True, True)
    assert all(w == 0 for w, _c in ran), ran
