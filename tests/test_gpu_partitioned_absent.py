"""Absent states inside `partition with` on the device NFA lanes, against the oracle bit for bit
(BASELINE config 5).

In a partitioned query the Scheduler's TreeMultimap keeps ONE partition instance per distinct
deadline (SchedulerState.compareTo == 0, Scheduler.java:77-97,364-366); the instance that fires is
the first in the key -> state HashMap's iteration order.  The device lanes fire independently, log
every firing, and when two instances shared a deadline at one tick the host replays the Scheduler
maps and defers the losers (nfa.hip NfaExec::flush).  The jittered stream never collides (each key
owns a residue of event time modulo the wait); the collision fixtures force the
exact replay.
"""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]
PART = ("@app:playback " + synth.STOCK_STREAM +
        " partition with (symbol of StockStream) begin @info(name='query1') ")

# BASELINE config 5 shape: logical `and` followed by an absent state, partitioned by key
ABSENT_AFTER_AND = PART + ("from every (e1=StockStream[price > 80] and e2=StockStream[volume > 900]) -> "
                           "not StockStream[price < 15] for 5 sec "
                           "select e1.symbol, e1.price as p1, e2.volume as v2 insert into Out; end;")
# absent start state with every (partitionCreated arms it at the key's first event)
EVERY_ABSENT_START = PART + ("from every not StockStream[price > 90] for 3 sec -> e2=StockStream[price < 20] "
                             "select e2.symbol, e2.price as p2 insert into Out; end;")
# logical absent (AbsentLogicalPreStateProcessor) in a partition
LOGICAL_ABSENT = PART + ("from every (e1=StockStream[price > 85] and not StockStream[volume > 950] for 2 sec) -> "
                         "e3=StockStream[price < 20] within 10 sec "
                         "select e1.symbol, e1.price as p1, e3.price as p3 insert into Out; end;")
LOGICAL_ABSENT_OR = PART + ("from every (e1=StockStream[price > 90] or not StockStream[volume > 980] for 2 sec) -> "
                            "e3=StockStream[price < 15] "
                            "select e1.price as p1, e3.price as p3 insert into Out; end;")


def rr_ticks(n, seed, k, start=0):
    return synth.stock_ticks_rr(n, seed, k, start=start)


def _run(ql, d, k, ncols, chunk=None):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]],
              batch=False, chunk=chunk, flush_each=chunk is not None)
    oo, go = o.raw_outputs(), g.raw_outputs()
    compare_raw(oo, go, ncols)
    return int(np.sum(go[0]["n_in"])), g


@pytest.mark.parametrize("n,k,chunk", [(30_000, 1000, None), (60_000, 1000, 20_000)])
def test_config5_absent_after_and_jittered(n, k, chunk):
    rows, g = _run(ABSENT_AFTER_AND, rr_ticks(n, synth.SEEDS[5], k), k, 3, chunk)
    assert rows > 0
    assert g.kernel_ms("nfa_exact_rounds") <= 0      # no shared deadlines: no replay needed


@pytest.mark.parametrize("par", [False, True])
@pytest.mark.parametrize("n,chunk", [(30_000, None), (45_000, 15_000)])
def test_config5_full_window_into_partitioned_absent(n, chunk, par, monkeypatch):
    """The whole config-5 app: `from StockStream#window.time(5 sec) ... insert into VolStream` runs on
    the window path at each push and its output chunks feed the partitioned pattern's absent state.  par: the
    host's thread-range paths for large pushes (the per-send clock and Scheduler ticks, window bookkeeping, the
    chained export's seqs) taken at this size (SG_HOST_PAR_MIN)."""
    if par:
        monkeypatch.setenv("SG_HOST_PAR_MIN", "64")
    rows, g = _run(synth.CONFIG5_FULL_QL, rr_ticks(n, synth.SEEDS[5], 1000), 1000, 3, chunk)
    assert g.path("window") == "window_agg"
    assert rows > 0
    assert g.kernel_ms("nfa_exact_rounds") <= 0


def test_every_absent_start_partitioned():
    rows, _ = _run(EVERY_ABSENT_START, rr_ticks(20_000, synth.SEEDS[5] + 1, 500), 500, 2)
    assert rows > 0


def test_logical_absent_partitioned():
    rows, _ = _run(LOGICAL_ABSENT, rr_ticks(20_000, synth.SEEDS[5] + 2, 400), 400, 2)
    assert rows > 0


def test_logical_absent_or_partitioned():
    rows, _ = _run(LOGICAL_ABSENT_OR, rr_ticks(20_000, synth.SEEDS[5] + 3, 400), 400, 2)
    assert rows > 0


# short waits over dense multi-key milliseconds: instances share deadlines at many ticks
SHARED_AND = ABSENT_AFTER_AND.replace("price > 80", "price > 60").replace("volume > 900", "volume > 600") \
    .replace("for 5 sec", "for 40 milliseconds")
SHARED_START = EVERY_ABSENT_START.replace("for 3 sec", "for 25 milliseconds")
SHARED_LOGICAL = LOGICAL_ABSENT.replace("for 2 sec", "for 30 milliseconds").replace("within 10 sec", "within 200 milliseconds")


@pytest.mark.parametrize("k,e,n", [(3, 2, 400), (16, 4, 1600), (40, 8, 2400)])
def test_shared_deadlines_fire_one_instance_per_tick(k, e, n):
    """Keys share deadlines (several keys per ms): the exact replay must reproduce which instance
    fires at each tick (the first in the Scheduler map's HashMap iteration order)."""
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 7, k=k, e=e)
    rows, g = _run(SHARED_AND, d, k, 3)
    assert rows > 0
    assert g.kernel_ms("nfa_exact_rounds") > 0


@pytest.mark.parametrize("ql", [SHARED_START, SHARED_LOGICAL], ids=["every_absent_start", "logical_absent"])
def test_shared_deadlines_other_shapes(ql):
    d = synth.stock_ticks(1500, seed=synth.SEEDS[5] + 9, k=12, e=3)
    rows, _ = _run(ql, d, 12, 2)
    assert rows > 0


@pytest.mark.parametrize("n", [3000, 12000])
def test_natural_collisions_random_keys(n):
    """Random keys at 10 events per ms (no jitter): instances share deadlines at most ticks.  Collisions that
    the replay's logs still describe exactly are resolved in the same round (nfa.hip resolve_first_collision),
    so the rounds stay far below the colliding ticks (r03: 2531 rounds for 10,000 events, one per tick)."""
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 11, k=1000, e=10)
    rows, g = _run(SHARED_AND, d, 1000, 3)
    assert rows > 0
    rounds = g.kernel_ms("nfa_exact_rounds")
    assert 0 < rounds < rows / 4, rounds
