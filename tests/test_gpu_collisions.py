"""Scheduler collisions at scale: the exact sweep (nfa.hip NfaExec::sweep).

In a partitioned query the Scheduler's TreeMultimap keeps ONE partition instance per distinct deadline at a tick
(SchedulerState.compareTo == 0, Scheduler.java:74-104,364-366): the first in the key -> state HashMap's iteration
order fires, the others are collected again at the next tick.  With random keys at 10 events per ms almost every
tick has such a collision.  The device lanes run independently and log their firings and map operations; the
host replays the maps window by window from a checkpoint (the sweep's base), defers the losers, and re-runs only
the deferred instances from the window's checkpoint.  Bar: bit-exact callbacks vs the oracle (which runs the
reference's Scheduler literally), a bounded event store across flushes, and snapshots that carry the base.
"""
import time

import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols
from test_gpu_partitioned_absent import SHARED_AND, STOCK_TYPES

pytestmark = pytest.mark.gpu

K = 1000


def _apps(ql=SHARED_AND, k=K):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    return o, g, gi


def _stream(n, seed=11, k=K):
    return synth.stock_ticks(n, seed=synth.SEEDS[5] + seed, k=k, e=10)


def test_sweep_and_round_replay_agree(monkeypatch):
    """The windowed sweep and the round-3 whole-app rounds (SG_NFA_REPLAY_ROUNDS) both match the oracle."""
    d = _stream(4000)
    for rounds_form in (False, True):
        if rounds_form:
            monkeypatch.setenv("SG_NFA_REPLAY_ROUNDS", "1")
        o, g, gi = _apps()
        feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], batch=False)
        compare_raw(o.raw_outputs(), g.raw_outputs(), 3)
        assert g.kernel_ms("nfa_exact_rounds") > 0


@pytest.mark.parametrize("window_ticks", ["1", "8", "4096"])
def test_sweep_window_sizes(monkeypatch, window_ticks):
    """Window size is a cost knob only: one tick, a few, or all of them."""
    monkeypatch.setenv("SG_NFA_SWEEP_TICKS", window_ticks)
    d = _stream(6000, seed=12)
    o, g, gi = _apps()
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], batch=False)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 3)


def test_sweep_base_across_flushes_compacts(monkeypatch):
    """Many flushes, each with collisions: every sweep starts at the previous one's end (its base), so the event
    store is compacted between flushes like any other NFA query's, and stays bounded."""
    monkeypatch.setenv("SG_NFA_COMPACT_MIN", "4000")
    n, chunk = 60_000, 3000
    d = _stream(n, seed=13)
    o, g, gi = _apps()
    peak, compacted = [0], [0]

    def after():
        peak[0] = max(peak[0], g.buffered("query1"))
        compacted[0] += g.kernel_ms("nfa_compacted_from") > 0

    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], batch=False,
              chunk=chunk, flush_each=True, after=after)
    compare_raw(o.raw_outputs(), g.raw_outputs(), 3)
    assert compacted[0] > 0
    assert peak[0] < n // 4, peak[0]


def test_snapshot_carries_sweep_base(monkeypatch):
    """A snapshot taken between colliding flushes restores into a fresh runtime that continues bit-exact (the
    base's Scheduler maps travel with it)."""
    monkeypatch.setenv("SG_NFA_COMPACT_MIN", "3000")
    n, chunk = 24_000, 2000
    d = _stream(n, seed=14)
    cols = [None, d["price"], d["volume"]]
    o, g, gi = _apps()
    cols[0] = gi[d["symbol"]]
    half = n // 2
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"][:half], [c[:half] for c in cols], batch=False,
              chunk=chunk, flush_each=True)
    first = g.raw_outputs()
    snap = g.snapshot()
    g2 = GpuApp(SHARED_AND); g2.add_query_callback("query1"); g2.start()
    assert np.array_equal(intern_symbols(g2, K), gi)
    g2.restore(snap)
    feed_both(o, g2, "StockStream", STOCK_TYPES, d["ts"][half:], [c[half:] for c in cols], batch=False,
              chunk=chunk, flush_each=True)
    second = g2.raw_outputs()
    both = tuple(np.concatenate([a, b]) if not isinstance(a, dict) else {x: np.concatenate([a[x], b[x]]) for x in a}
                 for a, b in zip(first, second))
    compare_raw(o.raw_outputs(), both, 3)


def test_one_million_colliding_events(monkeypatch):
    """a natural-collision config-5-shaped stream of 1M events (random keys, K = 1000, 10 events
    per ms, 40 ms absent wait), bit-exact vs the oracle, flushed every 100K events with a bounded store."""
    monkeypatch.setenv("SG_NFA_COMPACT_MIN", "150000")
    n, chunk = 1_000_000, 100_000
    d = _stream(n, seed=11)
    o, g, gi = _apps()
    peak, flush_s = [0], []
    t = [time.time()]

    def after():
        flush_s.append(time.time() - t[0])
        peak[0] = max(peak[0], g.buffered("query1"))
        t[0] = time.time()

    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], batch=False,
              chunk=chunk, flush_each=True, after=after)
    oo, go = o.raw_outputs(), g.raw_outputs()
    rows = compare_raw(oo, go, 3)
    print(f"\n1M colliding events: {sum(flush_s):.1f} s over {len(flush_s)} flushes (incl. the oracle's sends), "
          f"peak buffered {peak[0]}, last flush rounds {g.kernel_ms('nfa_exact_rounds'):.0f}")
    assert peak[0] < 400_000, peak[0]
