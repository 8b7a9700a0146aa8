"""Streaming shard protocol (shard mode 3: sg_query_shard_resolver, siddhi_amd/shard.py StreamingResolver) for a
partitioned query with absent states sharded by key, rehearsed on one GPU with one thread
per rank (shard.LocalGroup), against one oracle runtime over the whole stream, bit for bit.

Each rank runs as a single runtime: every flush from its settled base, the exact windowed sweep after a collision
(only deferred instances re-run, from the window's checkpoint), and the Scheduler-map questions -- a collision in
this run? the losers in this window? -- answered from every rank's logs.  Unlike the batch protocol
(test_gpu_shard_nfa.py, shard.settle_collisions), a settled window is never run again, so natural-collision
streams (random keys, several events per millisecond, a deadline shared at most ticks) settle, and the pushes can
be streamed: several pushes and flushes, no callback repeated (Scheduler.java:74-104, 364-366;
InputHandler.java:59-70)."""
import threading
import time

import numpy as np
import pytest

from siddhi_amd import shard, synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols
from test_gpu_partitioned_absent import SHARED_AND, SHARED_START
from test_gpu_shard_nfa import _key_hash, _oracle

pytestmark = pytest.mark.gpu


def _stream(ql, d, k, world, ids, nchunks):
    """Every rank pushes its share of each of nchunks global pushes (sg_push_shard) and flushes, concurrently
    (each flush waits inside the library for the other ranks' logs).  -> (merged outputs, resolvers)."""
    key = ids[d["symbol"]]
    grp = shard.LocalGroup(world, timeout=240)
    apps, res = [], []
    for r in range(world):
        g = GpuApp(ql)
        g.add_query_callback("query1")
        g.start()
        assert np.array_equal(intern_symbols(g, k), ids)
        assert g.path("query1") == "nfa"
        apps.append(g)
        res.append(shard.StreamingResolver(grp, g, "query1", _key_hash(g)))
    own = shard.owner(key, world)
    bounds = np.linspace(0, len(key), nchunks + 1).astype(int)
    outs = [[] for _ in range(world)]
    errs = []

    def run(r):
        grp.bind(r)
        try:
            for a, b in zip(bounds[:-1], bounds[1:]):
                idx = np.nonzero(own[a:b] == r)[0] + a
                cols = [key[idx], d["price"][idx], d["volume"][idx]]
                apps[r].push_shard("StockStream", d["ts"][idx], cols, idx, d["ts"][a:b], seq0=int(a), batch=False)
                outs[r].append(apps[r].raw_outputs())
        except BaseException as e:          # (a failed rank must not leave the others waiting at the barrier)
            errs.append(e)
            grp.bar.abort()
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for g in apps:
        g.close()
    if errs:
        raise errs[0]
    return shard.merge_outputs([p for o in outs for p in o]), res


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("nchunks", [1, 5])
@pytest.mark.parametrize("k,e,n", [(16, 4, 1600), (40, 8, 2400)])
def test_stream_shared_deadlines(world, nchunks, k, e, n):
    """Dense multi-key milliseconds with a 40 ms wait (collisions across ranks and within one), pushed and flushed
    in nchunks pieces: the single runtime's callbacks, none repeated."""
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 7, k=k, e=e)
    ref, ids = _oracle(SHARED_AND, d, k)
    merged, res = _stream(SHARED_AND, d, k, world, ids, nchunks)
    compare_raw(ref, merged, 3)
    assert sum(r.rounds for r in res) > 0              # (the fixture collides across ranks)


@pytest.mark.parametrize("world", [2, 4])
def test_stream_every_absent_start(world):
    d = synth.stock_ticks(1500, seed=synth.SEEDS[5] + 9, k=12, e=3)
    ref, ids = _oracle(SHARED_START, d, 12)
    merged, _ = _stream(SHARED_START, d, 12, world, ids, 6)
    compare_raw(ref, merged, 2)


@pytest.mark.parametrize("world", [2, 4])
def test_stream_natural_collisions_200k(world):
    """200,000 events over 1,000 random keys at 10 events per ms under the config-5 pattern shape (a 40 ms wait):
    a deadline is shared at most ticks.  The batch protocol did not settle this in 150 rounds
    (profiles/r05z_shard_natural_collision_rounds.log); the streaming one settles it window by window, 10 pushes
    and flushes, bit-exact, with one collided round per resolved batch of collisions."""
    n, k, e = 200_000, 1000, 10
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 11, k=k, e=e)
    ref, ids = _oracle(SHARED_AND, d, k)
    t0 = time.time()
    merged, res = _stream(SHARED_AND, d, k, world, ids, 10)
    dt = time.time() - t0
    compare_raw(ref, merged, 3)
    r0 = res[0]
    print(f"\nstreaming protocol, n={n} world={world}: {r0.rounds} collided rounds, {r0.windows} settled windows, "
          f"{r0.flushes} flushes, {dt:.1f} s, {len(merged[1])} rows")
    assert all(r.rounds == r0.rounds and r.windows == r0.windows for r in res)   # the ranks stayed in step
    assert r0.rounds > 0


@pytest.mark.parametrize("world", [2, 4])
def test_stream_host_thread_ranges(world, monkeypatch):
    """The host paths that split large pushes over thread ranges (the global send clock and its Scheduler ticks in
    sg_push_shard, the shard batch checks, the window and NFA bookkeeping) taken at test size (SG_HOST_PAR_MIN):
    the same callbacks as the single runtime."""
    monkeypatch.setenv("SG_HOST_PAR_MIN", "64")
    d = synth.stock_ticks(2400, seed=synth.SEEDS[5] + 7, k=40, e=8)
    ref, ids = _oracle(SHARED_AND, d, 40)
    merged, res = _stream(SHARED_AND, d, 40, world, ids, 5)
    compare_raw(ref, merged, 3)
    assert sum(r.rounds for r in res) > 0
