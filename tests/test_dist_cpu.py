"""Multi-process (world_size 2, gloo on CPU) check of the keyed routing step bench.py runs before the
keyed path on N GPUs: every event lands on the rank owning its key, per-key arrival order is kept
(source ranks own consecutive time ranges), and nothing is lost or duplicated."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import route_by_key
    from siddhi_amd import synth
    d = synth.stock_ticks_torch(n, seed=synth.SEEDS[4], k=997, e=10, start=rank * n, device="cpu")
    idx0 = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64)
    ts, sym, idx = route_by_key(dist, world, torch.device("cpu"), [d["ts"], d["symbol"], idx0], d["symbol"])
    # timestamps as 32-bit offsets over the wire: same result
    ts32, _s, idx2 = route_by_key(dist, world, torch.device("cpu"), [d["ts"], d["symbol"], idx0], d["symbol"],
                                  ts_base=synth.T0 - 5)
    assert ts32.dtype == torch.int64 and torch.equal(ts32, ts) and torch.equal(idx2, idx)
    out[rank] = (ts.numpy().copy(), sym.numpy().copy(), idx.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_keyed_routing_gloo(world):
    n = 5000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    seen = []
    for r in range(world):
        ts, sym, idx = out[r]
        assert np.all(sym % world == r)                 # owner of every key
        assert np.all(np.diff(idx) > 0)                 # global arrival order kept (hence per key)
        assert np.all(np.diff(ts) >= 0)                 # timestamps stay non-decreasing
        seen.append(idx)
    allidx = np.sort(np.concatenate(seen))
    assert np.array_equal(allidx, np.arange(world * n))


def _halo_worker(rank, world, port, n, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import halo_exchange
    from siddhi_amd import synth
    d = synth.stock_ticks_torch(n, seed=synth.SEEDS[1], k=1000, e=3, start=rank * n, device="cpu")
    idx = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64)
    halo = halo_exchange(dist, rank, world, torch.device("cpu"), [d["ts"], idx], d["ts"], 100)
    out[rank] = (d["ts"].numpy().copy(), halo[0].numpy().copy(), halo[1].numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_config1_halo_exchange_gloo(world):
    """Config 1's time-range split (bench.halo_exchange): rank g receives exactly the next rank's leading
    events with ts <= its first ts + W, in arrival order; the last rank receives none."""
    n = 4000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_halo_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    for r in range(world):
        _ts, hts, hidx = out[r]
        if r + 1 == world:
            assert len(hts) == 0
            continue
        nts = out[r + 1][0]
        want = np.nonzero(nts <= nts[0] + 100)[0]
        assert np.array_equal(hidx, (r + 1) * n + want)
        assert np.array_equal(hts, nts[want])
