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
    # bench.py routes a 4-B source position instead of the global index: rebuilt from the receive counts
    pos0 = torch.arange(n, dtype=torch.int32)
    _t, _s, pos = route_by_key(dist, world, torch.device("cpu"), [d["ts"], d["symbol"], pos0], d["symbol"])
    sc = torch.bincount((d["symbol"].to(torch.int64) % world), minlength=world)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    src = torch.repeat_interleave(torch.arange(world, dtype=torch.int64), rc)
    assert torch.equal(src * n + pos.to(torch.int64), idx)
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


def _gather_worker(rank, world, port, n, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from bench import route_by_key
    from oracle.pyoracle import OracleApp
    from siddhi_amd import shard, synth
    from synth_run import raw_matrix
    k = 300
    d = synth.stock_ticks_torch(n, seed=synth.SEEDS[4], k=k, e=5, start=rank * n, device="cpu")
    idx0 = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64)
    ts, sym, price, vol, idx = route_by_key(dist, world, torch.device("cpu"),
                                            [d["ts"], d["symbol"], d["price"], d["volume"], idx0], d["symbol"])
    # this rank's keyed runtime (the oracle stands in for the GPU on CPU): per-event sends
    o = OracleApp(synth.CONFIG4_QL)
    o.add_query_callback("query1")
    o.start()
    o.L.or_intern_range(o.h, b"S", k)
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [sym.numpy(), price.numpy(), vol.numpy()])
    o.send_columns(o.L.or_stream_index(o.h, b"StockStream"), ts.numpy(), raw, None, False)
    cbs, rts, rraw, rnul = o.raw_outputs()
    cbs["seq"] = idx.numpy()[o.callback_seq()]          # local arrival index -> global
    merged = shard.gather_merge(dist, (cbs, rts, rraw, rnul))
    if rank == 0:
        out["merged"] = merged
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_keyed_gather_merge_gloo(world):
    """Routing + per-rank keyed runtimes + gather to rank 0 + merge by arrival index == one runtime."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle.pyoracle import OracleApp
    from siddhi_amd import synth
    from synth_run import compare_raw, raw_matrix
    n = 20_000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gather_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    merged = out["merged"]
    d = synth.stock_ticks(world * n, seed=synth.SEEDS[4], k=300, e=5)
    o = OracleApp(synth.CONFIG4_QL)
    o.add_query_callback("query1")
    o.start()
    o.L.or_intern_range(o.h, b"S", 300)
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [d["symbol"], d["price"], d["volume"]])
    o.send_columns(o.L.or_stream_index(o.h, b"StockStream"), d["ts"], raw, None, False)
    ref = o.raw_outputs()
    assert len(ref[1]) > 1000
    compare_raw(ref, merged, 2)
