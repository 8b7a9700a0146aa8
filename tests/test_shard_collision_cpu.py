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


needs_golden = pytest.mark.skipif(not os.path.exists(GOLDEN), reason="recorded protocol fixture missing")


@needs_golden
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


@needs_golden
def test_one_process_driver_replays_recorded_protocol():
    z = dict(np.load(GOLDEN))
    world, rounds = int(z["world"]), int(z["rounds"])
    hk = dict(zip(z["hash_key"].tolist(), z["hash_val"].tolist()))
    apps = [_Replay(z, r) for r in range(world)]
    shard.settle_collisions(apps, "query1", lambda k: hk[int(k)])
    got = sorted(d for a in apps for d in a.defers)
    want = sorted((i, int(r), int(k), int(t), int(s)) for i in range(rounds) for r, k, t, s in z[f"defer_{i}"])
    assert got == want
