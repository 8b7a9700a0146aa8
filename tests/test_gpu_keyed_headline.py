"""Config 4 at the headline shape: K = 1M keys, E = 1000 events/ms, bit-exact against
the key-sharded oracle on all host cores (oracle/pyoracle.sharded_run, pinned by
tests/test_oracle_sharded.py).

The bench's timed stream has ~1 event per key per `within` window (1000 events/ms spread over 1M
keys), fills the 10-bit local-key field of the buckets and runs P = 1024 of them; this test
runs the same regime (same generator, seed, K and E) over its first 20M events and compares every
callback, row and float bit, for the chunk-sorted pipeline with its device order pass (keyed_chunks.hpp: the
path the bench times) and for the bucketed-tile matcher (keyed_tiles.hpp).  It also checks that the
device-resident bench path (push_device + flush_device) reports the same match count."""
import os

import numpy as np
import pytest

from oracle.pyoracle import sharded_run
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, raw_matrix

pytestmark = pytest.mark.gpu

K, E = 1_000_000, 1000


def _threads():
    return max(2, min(16, os.cpu_count() or 2))


@pytest.mark.parametrize("n", [20_000_000])
def test_config4_headline_shape_matches_sharded_oracle(n):
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.init()                      # bind the device in torch before the library does
    d = synth.stock_ticks(n, seed=synth.SEEDS[4], k=K, e=E)
    g = GpuApp(synth.CONFIG4_QL)
    g.add_query_callback("query1")
    g.start()
    base = g.intern("S0")
    for i in range(1, K):
        g.intern(f"S{i}")
    assert g.path("query1") == "keyed_followed_by"
    sym = (d["symbol"] + base).astype(np.int32)
    g.send_columns("StockStream", d["ts"], [sym, d["price"], d["volume"]], True)
    gout = g.raw_outputs()
    assert g.kernel_ms("k_kc_match") > 0 and g.kernel_ms("k_kt_order") > 0, "the chunk pipeline + order pass"
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [sym, d["price"], d["volume"]])
    t = _threads()
    oout, secs = sharded_run(synth.CONFIG4_QL, "StockStream", d["ts"], raw, d["symbol"] % t, t,
                             batch=True, symbols=K, shard_key=d["symbol"])
    compare_raw(oout, gout, 2)
    m = int(np.sum(gout[0]["n_in"]))
    assert m > n // 4
    print(f"{n} events, K={K}: {m} matches bit-exact; oracle {secs:.1f} s on {t} threads")

    # the bucketed-tile matcher on the same events: same callbacks
    os.environ["SG_KEYED_NO_CHUNKS"] = "1"
    try:
        gk = GpuApp(synth.CONFIG4_QL)
        gk.add_query_callback("query1")
        gk.start()
        for i in range(K):
            gk.intern(f"S{i}")
        gk.send_columns("StockStream", d["ts"], [sym, d["price"], d["volume"]], True)
        gkout = gk.raw_outputs()
        assert gk.kernel_ms("k_kt_match") > 0
        compare_raw(oout, gkout, 2)
        gk.close()
    finally:
        del os.environ["SG_KEYED_NO_CHUNKS"]

    # the bench's device-resident path on the same events: same match count
    g2 = GpuApp(synth.CONFIG4_QL)
    for i in range(K):
        g2.intern(f"S{i}")
    g2.start()
    ts = torch.from_numpy(d["ts"]).to(dev)
    sy = torch.from_numpy(sym).to(dev)
    pr = torch.from_numpy(d["price"]).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    g2.push_device("StockStream", n, ts.data_ptr(), [sy.data_ptr(), pr.data_ptr(), 0], hip_stream=stream)
    g2.flush_device(hip_stream=stream)
    torch.cuda.synchronize()
    assert g2.match_count("query1") == m
