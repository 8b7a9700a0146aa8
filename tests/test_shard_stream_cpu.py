"""CPU checks of the streaming shard protocol's driver side (siddhi_amd/shard.py resolve_window, StreamingResolver;
the GPU side with real rank runtimes is tests/test_gpu_shard_stream.py): a window's resolution from the maps at its
start equals the batch resolution over every log up to it, a settled window advances the maps, and the resolver's
questions go over torch.distributed (gloo, world_size 2) with each rank receiving exactly its own losers across
several flushes."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from siddhi_amd import shard
from test_shard_collision_cpu import _fires, _ops

# two ranks, keys 10 / 12 on rank 0 and 11 / 13 on rank 1; hashes put 10 and 11 in one bin (the later insertion
# heads the chain), 12 and 13 in another
H = {10: 5, 11: 5, 12: 6, 13: 6}
NOW = np.array([97, 98, 99, 100, 101, 102, 103, 104], np.int64)


def _window1():
    """Window 1 (ticks 0-2): every key arms a deadline (notifyAt), nothing collides."""
    ops = [_ops([(1, 0, 10, -1, 0, 0, 1, -1, 0), (3, 0, 12, -1, 0, 1, 1, -1, 0)]),
           _ops([(2, 0, 11, -1, 0, 0, 1, -1, 0), (4, 0, 13, -1, 0, 1, 1, -1, 0)])]
    fires = [_fires([(10, 90, 5, 2, 0, 0)]), _fires([(11, 91, 5, 2, 0, 0)])]
    return fires, ops


def _window2():
    """Window 2 (ticks 3-4): 10 and 11 share deadline 100 at tick 3, 12 and 13 deadline 101 at tick 4."""
    ops = [_ops([]), _ops([])]
    fires = [_fires([(10, 100, 6, 3, 0, 1), (12, 101, 7, 4, 0, 1)]),
             _fires([(11, 100, 6, 3, 0, 1), (13, 101, 7, 4, 0, 1)])]
    return fires, ops


def test_window_without_collision_advances_the_maps():
    fires, ops = _window1()
    losers, maps = shard.resolve_window(fires, ops, H.get, NOW, 40, {})
    assert losers == [] and maps is not None
    m = maps[0]
    assert m.size == 4
    assert m.rank(5, 11) < m.rank(5, 10)          # (11 inserted later: it heads bin 5's chain)


def test_window_from_the_base_equals_the_batch_resolution():
    """Resolving window 2 from the maps window 1 left gives what the batch protocol decides from every log."""
    f1, o1 = _window1()
    _, maps = shard.resolve_window(f1, o1, H.get, NOW, 40, {})
    f2, o2 = _window2()
    kept = repr(maps[0].tab)
    losers, adv = shard.resolve_window(f2, o2, H.get, NOW, 40, maps)
    assert adv is None and repr(maps[0].tab) == kept              # (a collided window leaves the base maps alone)
    fires = [np.concatenate([a, b]) for a, b in zip(f1, f2)]
    ops = [np.concatenate([a, b]) for a, b in zip(o1, o2)]
    assert losers == shard.resolve_collision(fires, ops, H.get, NOW, 40)
    assert losers == [(0, 10, 3, 0), (0, 12, 4, 0)]


class _FakeApp:
    def __init__(self):
        self.cb = None

    def shard_resolver(self, query, cb):
        self.cb = cb

    def sched_clock(self, query):
        return NOW, 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    app = _FakeApp()
    r = shard.StreamingResolver(dist, app, "query1", H.get)
    got = []
    f1, o1 = _window1()
    f2, o2 = _window2()
    for flush in range(5):                 # five flushes, each asking what a rank's runtime asks
        if flush == 0:                     # a run without a collision: no sweep
            got.append(app.cb(0, f1[rank], o1[rank]))
            continue
        got.append(app.cb(0, f2[rank], o2[rank]))           # the run collides at (tick 3, scheduler 0)
        if flush == 1:
            got.append(app.cb(1, f1[rank], o1[rank]))       # sweep window 1: settles
            got.append(app.cb(1, f2[rank], o2[rank]))       # window 2: losers on rank 0 only
            # after the re-run: rank 0's deferred instances fire one tick later, under their old heads
            rerun = _fires([(10, 100, 7, 4, 0, 1), (12, 101, 8, 5, 0, 1)]) if rank == 0 else f2[1]
            got.append(app.cb(1, rerun, o2[rank]))              # no collision left: the window settles
    out[rank] = (got, r.rounds, r.windows, r.flushes, sorted(r.maps))
    dist.barrier()
    dist.destroy_process_group()


def test_streaming_resolver_gloo_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    g0, g1 = out[0], out[1]
    # the same answers on both ranks, except the losers, which go to their owner
    assert g0[0][0] == g1[0][0] == (-1, [])
    assert g0[0][1] == g1[0][1] == ((3 << 8) | 0, [])
    assert g0[0][2] == g1[0][2] == (0, [])
    assert g0[0][3] == (1, [(10, 3, 0), (12, 4, 0)]) and g1[0][3] == (1, [])
    assert g0[0][4] == g1[0][4] == (0, [])
    for g in (g0, g1):
        assert g[1] == 1 and g[2] == 2 and g[3] == 5     # one collided round, two settled windows, five flushes
