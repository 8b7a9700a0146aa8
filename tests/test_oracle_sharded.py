"""The key-sharded multi-threaded oracle driver (oracle/pyoracle.sharded_run) equals one oracle app.

Partition instances never interact for patterns without absent states (PartitionStateHolder keys,
SURVEY §8e), so shards of disjoint keys run in parallel threads and their callbacks merge back by
the arrival index of the send that fired them.  This is what lets the headline-shape parity test
(K = 1M keys, tests/test_gpu_keyed_headline.py) and bench.py's multi-core CPU baseline use all host
cores."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp, sharded_run
from siddhi_amd import synth
from synth_run import compare_raw, intern_symbols, raw_matrix

TYPES = ["STRING", "FLOAT", "INT"]


@pytest.mark.parametrize("ql,k,e,batch", [
    (synth.CONFIG4_QL, 500, 50, True),
    (synth.CONFIG4_QL, 2000, 1000, False),
    (synth.CONFIG3_QL, 50, 1, True),
    (synth.CONFIG5_QL, 80, 2, False),
])
@pytest.mark.parametrize("threads", [2, 5])
def test_sharded_oracle_equals_single_app(ql, k, e, batch, threads):
    n = 60_000
    d = synth.stock_ticks(n, seed=synth.SEEDS[4] + threads, k=k, e=e)
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    ids = intern_symbols(o, k)
    raw = raw_matrix(TYPES, [ids[d["symbol"]], d["price"], d["volume"]])
    o.send_columns(o.L.or_stream_index(o.h, b"StockStream"), d["ts"], raw, None, batch)
    ref = o.raw_outputs()
    got, _secs = sharded_run(ql, "StockStream", d["ts"], raw, d["symbol"] % threads, threads,
                             batch=batch, symbols=k, shard_key=d["symbol"])
    assert len(ref[1]) > 0
    compare_raw(ref, got, 4)
