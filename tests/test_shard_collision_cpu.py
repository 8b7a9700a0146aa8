"""CPU checks of the cross-rank Scheduler collision protocol (siddhi_amd/shard.py; the GPU side is
tests/test_gpu_shard_nfa.py): the global HashMap replay on hand-built logs, and the exchange itself over
torch.distributed (gloo, world_size 2) replaying a protocol run recorded on the GPU
(tests/golden/sched_collision_w2.npz, made by tools/record_sched_logs.py: every round's per-rank firing /
notifyAt logs and the deferrals the one-process driver applied)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from siddhi_amd import shard
from siddhi_amd.runtime import SCHED_FIRE, SCHED_OP

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sched_collision_w2.npz")


def _fires(rows):
    a = np.zeros(len(rows), SCHED_FIRE)
    for i, (key, head, seq, tick, sched, empty) in enumerate(rows):
        a[i] = (key, head, seq, tick, sched, empty, 0)
    return a


def _ops(rows):
    a = np.zeros(len(rows), SCHED_OP)
    for i, (seq, head, key, tick, sub, pos, phase, kfire, ktarget) in enumerate(rows):
        a[i] = (seq, head, key, tick, sub, pos, phase, kfire, ktarget, 0)
    return a


def test_java_hash_matches_string_hashcode():
    # "S0".hashCode() = 31*'S' + '0' = 2621; HashMap.hash spreads h ^ (h >>> 16)
    assert shard.java_hash("S0") == 2621
    h = 0
    for ch in "partition-key-123":
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    assert shard.java_hash("partition-key-123") == h ^ (h >> 16)


def test_hashmap_order_bins_then_chain_and_resize():
    m = shard.JdkHashMap()
    m.touch(5, 100)
    m.touch(3, 200)
    m.touch(21, 300)            # bin 5 of 16, in front of key 100 in the chain
    assert m.rank(3, 200) < m.rank(21, 300) < m.rank(5, 100)
    for i in range(20):         # past 12 entries: 32 bins, 21 & 16 moves key 300 to bin 21
        m.touch(1000 + i, 1000 + i)
    assert m.rank(5, 100) < m.rank(21, 300)
    m.remove(5, 100)
    assert m.rank(5, 100) == (1 << 62,)


def test_first_collision_is_earliest_tick_then_scheduler():
    f = _fires([(1, 50, 7, 9, 0, 1), (2, 50, 7, 9, 0, 1),       # tick 9 sched 0 collides
                (3, 40, 5, 4, 1, 1), (4, 40, 5, 4, 1, 1),       # tick 4 sched 1 collides (earlier)
                (5, 40, 5, 4, 0, 1), (6, 41, 5, 4, 0, 1)])      # tick 4 sched 0: different heads
    assert shard.first_collision(f) == (4, 1)
    assert shard.first_collision(f[:2]) == (9, 0)
    assert shard.first_collision(f[4:]) is None


def _two_rank_logs(k0, k1, remove_first):
    """Keys k0 (rank 0) and k1 (rank 1) notify Scheduler 0 at their events (seq 1, seq 2) and both fire
    at tick 3 under head 100.  With remove_first, k0 had fired alone at tick 2 and left the map."""
    fires = [[], []]
    ops = [[(1, 0, k0, -1, 0, 0, 1, -1, 0)], [(2, 0, k1, -1, 0, 0, 1, -1, 0)]]
    if remove_first:
        fires[0].append((k0, 90, 3, 2, 0, 1))
        ops[0].append((4, 0, k0, -1, 0, 1, 1, -1, 0))     # k0 re-notifies at its next event (seq 4)
        fires[0].append((k0, 100, 5, 3, 0, 1))
        fires[1].append((k1, 100, 5, 3, 0, 1))
    else:
        fires[0].append((k0, 100, 5, 3, 0, 1))
        fires[1].append((k1, 100, 5, 3, 0, 1))
    return [_fires(f) for f in fires], [_ops(o) for o in ops]


def test_resolve_defers_the_instance_later_in_map_order():
    h = {10: 5, 11: 5}                       # one bin: the chain head (inserted last) iterates first
    fires, ops = _two_rank_logs(10, 11, False)
    assert shard.resolve_collision(fires, ops, h.get) == [(0, 10, 3, 0)]
    h = {10: 2, 11: 7}                       # bins 2 < 7
    assert shard.resolve_collision(fires, ops, h.get) == [(1, 11, 3, 0)]


def test_resolve_replays_removals_and_reinsertion():
    # k0 fired at tick 2 with an empty queue (removed), then re-inserted at seq 4: now the chain head
    h = {10: 5, 11: 5}
    fires, ops = _two_rank_logs(10, 11, True)
    assert shard.resolve_collision(fires, ops, h.get) == [(1, 11, 3, 0)]


def test_resolve_batches_collisions_the_logs_still_describe():
    """Two collisions one tick apart, other keys, other heads: with the ticks' clocks and the shortest wait the
    driver resolves both in one round (nfa.hip replay_maps' rule); without them only the first."""
    ops = [_ops([(1, 0, 10, -1, 0, 0, 1, -1, 0), (3, 0, 12, -1, 0, 1, 1, -1, 0)]),
           _ops([(2, 0, 11, -1, 0, 0, 1, -1, 0), (4, 0, 13, -1, 0, 1, 1, -1, 0)])]
    fires = [_fires([(10, 100, 5, 3, 0, 1), (12, 101, 6, 4, 0, 1)]),
             _fires([(11, 100, 5, 3, 0, 1), (13, 101, 6, 4, 0, 1)])]
    h = {10: 5, 11: 5, 12: 6, 13: 6}          # the later insertion heads each bin's chain and wins
    now = np.array([97, 98, 99, 100, 101, 102], np.int64)
    assert shard.resolve_collision(fires, ops, h.get) == [(0, 10, 3, 0)]
    assert shard.resolve_collision(fires, ops, h.get, now, 40) == [(0, 10, 3, 0), (0, 12, 4, 0)]
    # out of reach: the second tick's clock is past the first collision's clock plus the wait
    assert shard.resolve_collision(fires, ops, h.get, np.array([0, 0, 0, 100, 140, 141], np.int64), 40) == [(0, 10, 3, 0)]


def test_resolve_without_collision_is_empty():
    fires = [_fires([(10, 100, 5, 3, 0, 1)]), _fires([(11, 101, 5, 3, 0, 1)])]
    assert shard.resolve_collision(fires, [_ops([]), _ops([])], lambda k: 0) == []


# ---- the exchange over gloo, replaying the recorded GPU run ----

class _Replay:
    """A rank app serving the recorded logs round by round; records the deferrals it is given."""

    def __init__(self, z, rank):
        self.z, self.rank, self.i, self.defers = z, rank, -1, []

    def shard_mode(self, q, m):
        pass

    def raw_outputs(self):
        self.i += 1
        return ({"kind": np.zeros(0)}, None, None, None)

    def sched_fires(self, q):
        return self.z[f"fires_{self.i}_{self.rank}"]

    def sched_ops(self, q):
        return self.z[f"ops_{self.i}_{self.rank}"]

    def sched_defer(self, q, key, tick, sched):
        self.defers.append((self.i, self.rank, int(key), int(tick), int(sched)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = dict(np.load(GOLDEN))
    hk = dict(zip(z["hash_key"].tolist(), z["hash_val"].tolist()))
    app = _Replay(z, rank)
    shard.settle_collisions_dist(dist, app, "query1", lambda k: hk[int(k)])
    out[rank] = (app.i + 1, app.defers)
    dist.barrier()
    dist.destroy_process_group()


def test_recorded_protocol_fixture_is_committed():
    """The fixture is part of the tree (a missing one fails, it never skips the exchange tests)."""
    assert os.path.exists(GOLDEN), f"{GOLDEN} missing: run tools/record_sched_logs.py on a GPU box"


def test_collision_exchange_gloo_replays_recorded_protocol():
    z = dict(np.load(GOLDEN))
    world, rounds = int(z["world"]), int(z["rounds"])
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gloo_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    want = [(i, int(r), int(k), int(t), int(s)) for i in range(rounds) for r, k, t, s in z[f"defer_{i}"]]
    assert sum(len(z[f"defer_{i}"]) for i in range(rounds)) > 10        # the fixture really collides
    assert any(len(z[f"fires_{i}_1"]) and len(z[f"defer_{i}"]) and np.any(z[f"defer_{i}"][:, 0] == 1)
               for i in range(rounds))                                   # ... and defers on both ranks
    for r in range(world):
        nrounds, defers = out[r]
        assert nrounds == rounds
        assert sorted(defers) == sorted(d for d in want if d[1] == r)


def test_one_process_driver_replays_recorded_protocol():
    z = dict(np.load(GOLDEN))
    world, rounds = int(z["world"]), int(z["rounds"])
    hk = dict(zip(z["hash_key"].tolist(), z["hash_val"].tolist()))
    apps = [_Replay(z, r) for r in range(world)]
    shard.settle_collisions(apps, "query1", lambda k: hk[int(k)])
    got = sorted(d for a in apps for d in a.defers)
    want = sorted((i, int(r), int(k), int(t), int(s)) for i in range(rounds) for r, k, t, s in z[f"defer_{i}"])
    assert got == want


# ---- bench.py's config-5 step on two gloo ranks: routing + the protocol with the tensor collision test ----

def _bench5_worker(rank, world, port, out):
    """What bench.step5_sharded does on each rank, with the rank app replaced by the recorded logs of the same
    fixture: route the rank's time range of the stream to the key owners (bench.route_by_key), all-gather the
    global send timestamps, then settle with the first round's collision test done as a tensor exchange."""
    import sys
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import route_by_key
    from siddhi_amd import synth
    z = dict(np.load(GOLDEN))
    hk = dict(zip(z["hash_key"].tolist(), z["hash_val"].tolist()))
    # the fixture's stream (tools/record_sched_logs.py): keys are dictionary ids 0..K-1 of "S0".."S{K-1}"
    d = synth.stock_ticks(int(z["n"]), seed=synth.SEEDS[5] + 7, k=int(z["k"]), e=int(z["e"]))
    n = len(d["ts"]) // world
    lo = rank * n
    cpu = torch.device("cpu")
    key = torch.from_numpy(z["key_of_symbol"][d["symbol"]][lo:lo + n].astype(np.int32))
    ts = torch.from_numpy(d["ts"][lo:lo + n])
    pos = torch.arange(n, dtype=torch.int32)
    rts, rkey, rpos = route_by_key(dist, world, cpu, [ts, key, pos], key, ts_base=int(d["ts"][0]))
    sc = torch.bincount(key.to(torch.int64) % world, minlength=world)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    seq = torch.repeat_interleave(torch.arange(world, dtype=torch.int64), rc) * n + rpos.to(torch.int64)
    gl = [torch.empty_like(ts) for _ in range(world)]
    dist.all_gather(gl, ts)
    gts = torch.cat(gl)
    app = _Replay(z, rank)
    shard.settle_collisions_dist(dist, app, "query1", lambda k: hk[int(k)], device=cpu,
                                 collect=lambda: app.raw_outputs()[0])
    out[rank] = (seq.numpy().copy(), rkey.numpy().copy(), rts.numpy().copy(), gts.numpy().copy(), app.i + 1,
                 app.defers)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_config5_step_gloo_routes_and_settles():
    from siddhi_amd import synth
    z = dict(np.load(GOLDEN))
    world, rounds = int(z["world"]), int(z["rounds"])
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench5_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    d = synth.stock_ticks(int(z["n"]), seed=synth.SEEDS[5] + 7, k=int(z["k"]), e=int(z["e"]))
    key = z["key_of_symbol"][d["symbol"]]
    want = [(i, int(r), int(k), int(t), int(s)) for i in range(rounds) for r, k, t, s in z[f"defer_{i}"]]
    for r in range(world):
        seq, rkey, rts, gts, nrounds, defers = out[r]
        idx = shard.route_host(key, world)[r]           # the recorded run's push on rank r
        assert np.array_equal(seq, idx) and np.array_equal(rkey, key[idx]) and np.array_equal(rts, d["ts"][idx])
        assert np.array_equal(gts, d["ts"])             # every rank ticks over every global send
        assert nrounds == rounds                        # the tensor test replaces round 0's object exchange
        assert sorted(defers) == sorted(x for x in want if x[1] == r)


def _any_collision_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cases = {
        "cross": [_fires([(1, 50, 7, 9, 0, 1)]), _fires([(2, 50, 7, 9, 0, 1)])],
        "local": [_fires([(1, 50, 7, 9, 0, 1), (3, 50, 7, 9, 0, 1)]), _fires([])],
        "none": [_fires([(1, 50, 7, 9, 0, 1), (3, 51, 7, 9, 0, 1)]), _fires([(2, 50, 7, 9, 1, 1)])],
        "empty": [_fires([]), _fires([])],
    }
    out[rank] = {c: shard.any_collision_dist(dist, f[rank]) for c, f in cases.items()}
    dist.barrier()
    dist.destroy_process_group()


def test_any_collision_dist_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_any_collision_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert out[r] == {"cross": True, "local": True, "none": False, "empty": False}
