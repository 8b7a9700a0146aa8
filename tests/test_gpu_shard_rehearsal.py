"""One-GPU rehearsal of multi-GPU keyed sharding (siddhi_amd/shard.py): the stream is split
into G contiguous time ranges, each event is routed to the rank owning its key (key % G) with its global
arrival index, every rank runs the keyed path on its events (its own runtime), and the ranks' callbacks
merged by arrival index must equal one runtime over the whole stream, bit for bit (the oracle)."""
import numpy as np
import pytest

from oracle.pyoracle import sharded_run
from siddhi_amd import shard, synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, raw_matrix

pytestmark = pytest.mark.gpu

K, E, N = 20_000, 200, 2_000_000


@pytest.fixture(scope="module")
def stream():
    d = synth.stock_ticks(N, seed=synth.SEEDS[4] + 11, k=K, e=E)
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [d["symbol"], d["price"], d["volume"]])
    ref, _ = sharded_run(synth.CONFIG4_QL, "StockStream", d["ts"], raw, d["symbol"] % 8, 8, batch=True,
                         symbols=K, shard_key=d["symbol"])
    return d, ref


@pytest.mark.parametrize("world", [2, 4, 8])
def test_keyed_shards_merge_to_single_runtime_order(stream, world):
    d, ref = stream
    parts = []
    for r, idx in enumerate(shard.route_host(d["symbol"], world)):
        g = GpuApp(synth.CONFIG4_QL)
        g.add_query_callback("query1")
        g.start()
        for i in range(K):
            g.intern(f"S{i}")
        assert g.path("query1") == "keyed_followed_by"
        assert np.all(d["symbol"][idx] % world == r)
        g.send_columns("StockStream", d["ts"][idx], [d["symbol"][idx], d["price"][idx], d["volume"][idx]], True,
                       seq=idx)
        parts.append(g.raw_outputs())
        g.close()
    merged = shard.merge_outputs(parts)
    compare_raw(ref, merged, 2)
    assert len(merged[1]) > N // 4
