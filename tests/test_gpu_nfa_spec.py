"""Speculative time segments of the NFA lanes (nfa.hip NfaExec::run_spec), against the oracle bit for bit.

A key's timeline is cut into segments run in parallel; each segment after the first starts from a newly
created instance, replays the events before it without emitting, and keeps its records only when its state
then equals (in canonical form) the state the previous segment ended with.  Otherwise the key re-runs from
its last verified state.  The tests force segmentation (SG_NFA_SPEC=1) with short segments so that both
outcomes occur: long warm-ups that verify, and warm-ups too short to rebuild a state (re-runs).  The shapes
include state that never converges (a one-shot start: `e1 -> e2` without `every`), so the re-run path decides
those keys entirely.  Several flushes per run check that the verified end state is carried to the next flush."""
import os

import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, feed_both, intern_symbols
from test_gpu_nfa_configs import CONFIG3_EVERY, CONFIG3_LITERAL, CONFIG5_LOGICAL, PART

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]

PATTERN_COUNT = PART + ("from every e1=StockStream[price > 30] -> e2=StockStream[price > e1.price]<2:4> -> "
                        "e3=StockStream[price < e2[last].price] within 2 sec "
                        "select e1.symbol, e1.price as p1, e2[last].price as p2, e3.price as p3 insert into Out; end;")
PATTERN_EVERY = PART + ("from every e1=StockStream[price > 60] -> e2=StockStream[price > e1.price] "
                        "-> e3=StockStream[price < 30] within 3 sec "
                        "select e1.price as p1, e2.price as p2, e3.price as p3 insert into Out; end;")
ONE_SHOT = PART + ("from e1=StockStream[price > 90] -> e2=StockStream[price > e1.price] "
                   "select e1.price as p1, e2.price as p2 insert into Out; end;")
UNPARTITIONED = synth.STOCK_STREAM + (
    "@info(name='query1') from every e1=StockStream, e2=StockStream[price > e1.price]+, "
    "e3=StockStream[price < e2[last].price] select e1.price as p1, e2[last].price as p2, e3.price as p3 "
    "insert into Out;")


@pytest.fixture
def spec_env():
    keys = ("SG_NFA_SPEC", "SG_NFA_SEG", "SG_NFA_WARM")
    old = {k: os.environ.get(k) for k in keys}

    def set_(seg, warm):
        os.environ["SG_NFA_SPEC"] = "1"
        os.environ["SG_NFA_SEG"] = str(seg)
        os.environ["SG_NFA_WARM"] = str(warm)
    yield set_
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _run(ql, n, seed, k, ncols, chunk=None):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    d = synth.stock_ticks(n, seed=seed, k=k, e=1)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], chunk=chunk)
    oo, go = o.raw_outputs(), g.raw_outputs()
    compare_raw(oo, go, ncols)
    st = {x: g.kernel_ms(x) for x in ("nfa_spec_tasks", "nfa_spec_rerun_tasks", "nfa_spec_rerun_keys",
                                     "nfa_spec_repaired_tasks")}
    return int(np.sum(go[0]["n_in"])), st


@pytest.mark.parametrize("seg,warm", [(64, 32), (64, 2), (200, 96)])
def test_spec_config3_every(spec_env, seg, warm):
    spec_env(seg, warm)
    rows, st = _run(CONFIG3_EVERY, 60_000, synth.SEEDS[3], 40, 5)
    assert rows > 0 and st["nfa_spec_tasks"] > 40


def test_spec_config3_every_rerun_path(spec_env):
    # a warm-up of one event cannot rebuild the rising-run partials: most segments re-run
    spec_env(32, 1)
    rows, st = _run(CONFIG3_EVERY, 30_000, synth.SEEDS[3] + 7, 20, 5)
    assert rows > 0 and st["nfa_spec_rerun_tasks"] > 0


def test_spec_config3_literal_never_converges(spec_env):
    spec_env(64, 32)
    rows, _ = _run(CONFIG3_LITERAL, 40_000, synth.SEEDS[3], 40, 4)
    assert 0 < rows <= 40


@pytest.mark.parametrize("ql,ncols", [(PATTERN_COUNT, 4), (PATTERN_EVERY, 3), (CONFIG5_LOGICAL, 4), (ONE_SHOT, 2)])
def test_spec_pattern_shapes(spec_env, ql, ncols):
    spec_env(128, 64)
    _run(ql, 50_000, synth.SEEDS[5] + 3, 25, ncols)


def test_spec_multiple_flushes(spec_env):
    # the verified (or re-run) end state of each key carries into the next flush
    spec_env(64, 48)
    rows, _ = _run(CONFIG3_EVERY, 90_000, synth.SEEDS[3] + 1, 30, 5, chunk=20_011)
    assert rows > 0


def test_spec_unpartitioned(spec_env):
    spec_env(256, 64)
    rows, st = _run(UNPARTITIONED, 40_000, synth.SEEDS[3] + 2, 100, 3)
    assert rows > 0 and st["nfa_spec_tasks"] > 100


@pytest.mark.parametrize("chunks", [1, 3])
def test_device_push_matches_oracle(spec_env, chunks):
    """sg_push_device into the NFA path (the bench's config-3 ingest): device-to-device event store, host
    instance bookkeeping from the partition keys; per chunk against the oracle's batch sends."""
    import torch
    spec_env(256, 32)
    k, n = 40, 60_000
    d = synth.stock_ticks(n, seed=synth.SEEDS[3] + 5, k=k, e=1)
    o = OracleApp(CONFIG3_EVERY); o.add_query_callback("query1"); o.start()
    g = GpuApp(CONFIG3_EVERY); g.add_query_callback("query1"); g.start()
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    dev = torch.device("cuda", 0)
    sym = gi[d["symbol"]]
    si = o.L.or_stream_index(o.h, b"StockStream")
    from synth_run import raw_matrix
    raw = raw_matrix(STOCK_TYPES, [sym, d["price"], d["volume"]])
    stream = torch.cuda.current_stream(dev).cuda_stream
    bounds = np.linspace(0, n, chunks + 1).astype(int)
    for a, b in zip(bounds[:-1], bounds[1:]):
        o.send_columns(si, d["ts"][a:b], raw[a:b], None, True)
        ts = torch.from_numpy(d["ts"][a:b]).to(dev)
        cols = [torch.from_numpy(np.ascontiguousarray(c[a:b])).to(dev) for c in (sym, d["price"], d["volume"])]
        torch.cuda.synchronize()
        g.push_device("StockStream", b - a, ts.data_ptr(), [c.data_ptr() for c in cols], hip_stream=stream, batch=True)
        g.flush()                   # one flush per chunk: the spec run's end states carry into the next
    compare_raw(o.raw_outputs(), g.raw_outputs(), 5)


# ---- absent states: Scheduler ticks inside segments (the end state is taken before the ticks that follow a
# segment's last event; the next segment runs them), the Scheduler queues in the canonical form, firings of
# unverified segments dropped before the collision check
from test_gpu_partitioned_absent import (ABSENT_AFTER_AND, EVERY_ABSENT_START, LOGICAL_ABSENT,  # noqa: E402
                                         LOGICAL_ABSENT_OR, SHARED_AND, rr_ticks)

UNPART_ABSENT = ("@app:playback " + synth.STOCK_STREAM +
                 " @info(name='query1') from every e1=StockStream[price > 96] -> not StockStream[price < 11] "
                 "for 500 milliseconds select e1.symbol, e1.price as p1 insert into Out;")


def _run_abs(ql, d, k, ncols, chunk=None):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]],
              batch=False, chunk=chunk, flush_each=chunk is not None)
    oo, go = o.raw_outputs(), g.raw_outputs()
    compare_raw(oo, go, ncols)
    return int(np.sum(go[0]["n_in"])), g


@pytest.mark.parametrize("ql,ncols", [(ABSENT_AFTER_AND, 3), (EVERY_ABSENT_START, 2), (LOGICAL_ABSENT, 2),
                                      (LOGICAL_ABSENT_OR, 2)],
                         ids=["absent_after_and", "every_absent_start", "logical_absent", "logical_absent_or"])
@pytest.mark.parametrize("seg,warm", [(64, 32), (32, 2)])
def test_spec_partitioned_absent(spec_env, ql, ncols, seg, warm):
    spec_env(seg, warm)
    rows, g = _run_abs(ql, rr_ticks(24_000, synth.SEEDS[5] + 4, 40), 40, ncols)
    assert g.kernel_ms("nfa_spec_tasks") > 40


def test_spec_config5_full_app(spec_env):
    spec_env(64, 32)
    # (200 round-robin keys: 25 events per key in the 5-second wait, inside the Scheduler queue's 64 runs)
    _run_abs(synth.CONFIG5_FULL_QL, rr_ticks(40_000, synth.SEEDS[5], 200), 200, 3, chunk=10_000)


def test_spec_shared_deadlines_then_exact_replay(spec_env):
    # segments run first; the firings left after dropping unverified segments collide, so the exact replay
    # (without segments) decides
    spec_env(16, 8)
    d = synth.stock_ticks(1600, seed=synth.SEEDS[5] + 7, k=16, e=4)
    rows, g = _run_abs(SHARED_AND, d, 16, 3)
    assert rows > 0 and g.kernel_ms("nfa_exact_rounds") > 0


def test_spec_unpartitioned_absent(spec_env):
    spec_env(256, 64)
    rows, g = _run_abs(UNPART_ABSENT, synth.stock_ticks(20_000, seed=synth.SEEDS[5] + 11, k=100, e=1), 100, 2)
    assert rows > 0


# ---- round 6: repair rounds, pools in global memory in blocks of 64 lanes, small scratch pools ----

@pytest.mark.parametrize("ql,ncols,absent", [(CONFIG3_EVERY, 5, False), (ABSENT_AFTER_AND, 3, True)],
                         ids=["config3_every", "absent_after_and"])
def test_spec_repair_rounds(spec_env, monkeypatch, ql, ncols, absent):
    """Warm-ups too short to rebuild every segment's state: the repair rounds re-run just the unverified segments
    from their keys' true states (NfaExec::run_spec), bit-exact; with SG_NFA_REPAIR_ROUNDS=0 the same keys re-run
    whole (the pre-round-6 path), bit-exact too."""
    spec_env(48, 3)
    seen = {}
    for rounds in ("8", "0"):
        monkeypatch.setenv("SG_NFA_REPAIR_ROUNDS", rounds)
        if absent:
            _, g = _run_abs(ql, rr_ticks(24_000, synth.SEEDS[5] + 9, 40), 40, ncols)
            st = {x: g.kernel_ms(x) for x in ("nfa_spec_repaired_tasks", "nfa_spec_rerun_tasks")}
        else:
            _, st = _run(ql, 40_000, synth.SEEDS[3] + 9, 30, ncols)
            g = None
        seen[rounds] = st
    assert seen["8"]["nfa_spec_repaired_tasks"] > 0
    assert seen["0"]["nfa_spec_rerun_tasks"] > 0


@pytest.mark.parametrize("ql,ncols,absent", [(CONFIG3_EVERY, 5, False), (CONFIG5_LOGICAL, 4, False),
                                             (ABSENT_AFTER_AND, 3, True), (LOGICAL_ABSENT, 2, True)],
                         ids=["config3_every", "config5_logical", "absent_after_and", "logical_absent"])
def test_spec_blocked_global_pools(spec_env, monkeypatch, ql, ncols, absent):
    """A launch of many speculative lanes keeps its pools in global memory, the scratch pools in blocks of 64 lanes
    (nfa_block_view); forced here at small sizes by SG_NFA_LDS_MAX_LANES, bit-exact vs the oracle."""
    spec_env(48, 32)
    monkeypatch.setenv("SG_NFA_LDS_MAX_LANES", "16")
    if absent:
        _, g = _run_abs(ql, rr_ticks(30_000, synth.SEEDS[5] + 13, 40), 40, ncols)
        assert g.kernel_ms("nfa_spec_blocked") == 1
    else:
        rows, _ = _run(ql, 60_000, synth.SEEDS[3] + 13, 40, ncols)
        assert rows > 0


def test_spec_small_scratch_pools_overflow(spec_env, monkeypatch):
    """Scratch pools too small for the stream: an overflowing segment fails verification and is repaired (and the
    pools grow for the next flush), never a wrong record."""
    spec_env(64, 32)
    monkeypatch.setenv("SG_NFA_SPEC_CAPS", "4,8,4")
    rows, _ = _run(CONFIG3_EVERY, 50_000, synth.SEEDS[3] + 17, 30, 5, chunk=12_503)
    assert rows > 0
