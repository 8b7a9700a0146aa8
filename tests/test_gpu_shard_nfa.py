"""One-GPU rehearsal of BASELINE configs 3 and 5 sharded by partition key over 1/2/4/8 ranks (SURVEY §8e,
siddhi_amd/shard.py), against one oracle runtime over the whole stream, bit for bit.

Every rank is its own runtime holding the keys it owns (key % world).  Config 3 has no clock state: each
rank sends its events with their global arrival seqs and the merge by seq restores the single-runtime
callback order.  Config 5 (playback, an absent state under `partition with`) follows the clock: every
rank pushes its share of each global send through sg_push_shard, so all ranks see the same Scheduler
ticks; timer callbacks merge by (seq, scheduler, deadline).  Instances of keys on different ranks that
share a deadline at one tick collide (Scheduler.java:77-97 keeps one SchedulerState per deadline): the
protocol of shard.settle_collisions replays the single runtime's key -> state HashMap over all ranks'
firing / notifyAt logs and defers the losers on their owner ranks.  The jittered stream never collides;
the dense multi-key fixtures collide at many ticks, across ranks and within one."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import shard, synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix
from test_gpu_partitioned_absent import SHARED_AND, SHARED_START

pytestmark = pytest.mark.gpu

STOCK_TYPES = ["STRING", "FLOAT", "INT"]


def _oracle(ql, d, k, batch=False):
    o = OracleApp(ql)
    o.add_query_callback("query1")
    o.start()
    ids = intern_symbols(o, k)
    si = o.L.or_stream_index(o.h, b"StockStream")
    o.send_columns(si, d["ts"], raw_matrix(STOCK_TYPES, [ids[d["symbol"]], d["price"], d["volume"]]), None, batch)
    return o.raw_outputs(), ids


def _ranks(ql, d, k, world, ids, clock):
    """The rank apps after each pushed its share; `clock`: push through sg_push_shard (global ticks)."""
    key = ids[d["symbol"]]
    apps = []
    for r, idx in enumerate(shard.route_host(key, world)):
        g = GpuApp(ql)
        g.add_query_callback("query1")
        g.start()
        assert np.array_equal(intern_symbols(g, k), ids)
        assert g.path("query1") == "nfa"
        assert np.all(key[idx] % world == r)
        cols = [key[idx], d["price"][idx], d["volume"][idx]]
        if clock:
            g.push_shard("StockStream", d["ts"][idx], cols, idx, d["ts"], batch=False)
        else:
            g.send_columns("StockStream", d["ts"][idx], cols, False, seq=idx)
        apps.append(g)
    return apps


def _key_hash(app):
    return lambda key: shard.java_hash(app.string(int(key)))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_config3_shards(world):
    k = 1000
    d = synth.stock_ticks(60_000, seed=synth.SEEDS[3], k=k)
    ref, ids = _oracle(synth.CONFIG3_QL, d, k)
    apps = _ranks(synth.CONFIG3_QL, d, k, world, ids, clock=False)
    merged = shard.merge_outputs([a.raw_outputs() for a in apps])
    compare_raw(ref, merged, 4)
    assert len(merged[1]) > 0
    for a in apps:
        a.close()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_config5_full_shards_jittered(world):
    """The whole config-5 app (upstream time window into the partitioned absent pattern) on the jittered
    stream: no deadline is shared, so the protocol settles after the first run."""
    k = 1000
    d = synth.stock_ticks_rr(30_000, synth.SEEDS[5], k)
    ref, ids = _oracle(synth.CONFIG5_FULL_QL, d, k)
    apps = _ranks(synth.CONFIG5_FULL_QL, d, k, world, ids, clock=True)
    parts = shard.settle_collisions(apps, "query1", _key_hash(apps[0]))
    merged = shard.merge_outputs(parts)
    compare_raw(ref, merged, 3)
    assert len(merged[1]) > 0
    for a in apps:
        a.close()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("k,e,n", [(3, 2, 400), (16, 4, 1600), (40, 8, 2400)])
def test_config5_shared_deadline_collisions_across_shards(world, k, e, n):
    """Dense multi-key milliseconds with a 40 ms wait: instances of keys on different ranks share
    deadlines; the winner at each tick must be the single runtime's (HashMap iteration order)."""
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 7, k=k, e=e)
    ref, ids = _oracle(SHARED_AND, d, k)
    apps = _ranks(SHARED_AND, d, k, world, ids, clock=True)
    parts = shard.settle_collisions(apps, "query1", _key_hash(apps[0]))
    compare_raw(ref, shard.merge_outputs(parts), 3)
    for a in apps:
        a.close()


@pytest.mark.parametrize("world", [2, 4])
def test_every_absent_start_collisions_across_shards(world):
    d = synth.stock_ticks(1500, seed=synth.SEEDS[5] + 9, k=12, e=3)
    ref, ids = _oracle(SHARED_START, d, 12)
    apps = _ranks(SHARED_START, d, 12, world, ids, clock=True)
    parts = shard.settle_collisions(apps, "query1", _key_hash(apps[0]))
    compare_raw(ref, shard.merge_outputs(parts), 2)
    for a in apps:
        a.close()


def test_protocol_resolves_several_collisions_per_round(monkeypatch):
    """With the ticks' clocks (sg_query_sched_clock) a protocol round resolves every collision its logs still
    describe, not only the first: the same output as one per round, in fewer rounds."""
    k, e, n = 40, 8, 2400
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 7, k=k, e=e)
    ref, ids = _oracle(SHARED_AND, d, k)
    rounds = []
    for one in (False, True):
        if one:
            monkeypatch.setenv("SG_SHARD_ONE_PER_ROUND", "1")
        apps = _ranks(SHARED_AND, d, k, 4, ids, clock=True)
        parts = shard.settle_collisions(apps, "query1", _key_hash(apps[0]))
        compare_raw(ref, shard.merge_outputs(parts), 3)
        rounds.append(shard.last_rounds)
        for a in apps:
            a.close()
    print(f"\nprotocol rounds: batched {rounds[0]}, one per round {rounds[1]}")
    assert rounds[0] < rounds[1], rounds


def test_collision_fixture_needs_the_protocol():
    """Without the protocol (each rank resolving only its own keys) the fixture's output differs: the
    collisions it covers really cross ranks."""
    k, e, n = 16, 4, 1600
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 7, k=k, e=e)
    ref, ids = _oracle(SHARED_AND, d, k)
    apps = _ranks(SHARED_AND, d, k, 2, ids, clock=True)
    naive = shard.merge_outputs([a.raw_outputs() for a in apps])
    with pytest.raises(AssertionError):
        compare_raw(ref, naive, 3)
    for a in apps:
        a.close()

