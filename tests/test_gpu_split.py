"""Multi-GPU split of the unkeyed config-1 pattern (sg_set_halo), rehearsed on one GPU: the
stream is cut into contiguous time ranges, each range runs on its own runtime with the next ranges'
events within W appended as halo (they complete the range's partials but start none), and the ranges'
outputs merged by trigger equal the oracle's output over the whole stream, bit for bit."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

TYPES = ["STRING", "FLOAT", "INT"]


def _split_run(ql, n, k, e, ranks, within, ncols):
    d = synth.stock_ticks(n, seed=synth.SEEDS[1], k=k, e=e)
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    oi = intern_symbols(o, k)
    si = o.L.or_stream_index(o.h, b"StockStream")
    o.send_columns(si, d["ts"], raw_matrix(TYPES, [oi[d["symbol"]], d["price"], d["volume"]]), None, True)
    want = o.raw_outputs()
    bounds = np.linspace(0, n, ranks + 1).astype(np.int64)
    per_ts = {}                                   # trigger ts (unique per event here) -> [(n_in, rows)]
    for r in range(ranks):
        lo, hi = bounds[r], bounds[r + 1]
        hend = int(np.searchsorted(d["ts"], d["ts"][hi - 1] + within, side="right")) if hi < n else n
        g = GpuApp(ql); g.add_query_callback("query1"); g.start()
        gi = intern_symbols(g, k)
        cols = [gi[d["symbol"][lo:hend]], d["price"][lo:hend], d["volume"][lo:hend]]
        g.send_columns("StockStream", d["ts"][lo:hend], cols, True)
        g.set_halo("StockStream", hend - hi)
        cbs, ts, raw, nul = g.raw_outputs()
        row = 0
        for c in range(len(cbs["ts"])):
            m = int(cbs["n_in"][c])
            per_ts.setdefault(int(cbs["ts"][c]), []).append((raw[row:row + m], nul[row:row + m], ts[row:row + m]))
            row += m
    keys = sorted(per_ts)
    raws = [x[0] for t in keys for x in per_ts[t]]
    nuls = [x[1] for t in keys for x in per_ts[t]]
    tss = [x[2] for t in keys for x in per_ts[t]]
    cb = dict(kind=np.zeros(len(keys), np.int32), target=np.zeros(len(keys), np.int32),
              ts=np.array(keys, np.int64), n_in=np.array([sum(len(x[0]) for x in per_ts[t]) for t in keys], np.int32),
              n_rm=np.zeros(len(keys), np.int32))
    w = want[2].shape[1]
    got = (cb, np.concatenate(tss) if tss else np.empty(0, np.int64),
           np.concatenate(raws)[:, :w] if raws else np.empty((0, w), np.int64),
           np.concatenate(nuls)[:, :w] if nuls else np.empty((0, w), np.uint8))
    compare_raw(want, got, ncols)
    assert len(keys) > 100


@pytest.mark.parametrize("n,ranks", [(60_000, 2), (90_000, 3), (200_000, 8)])
def test_config1_time_split_with_halo_matches_single_stream(n, ranks):
    _split_run(synth.CONFIG1_QL, n, 1000, 1, ranks, 1000, 2)


def test_config1_halo_generic_predicate_path():
    """The bytecode (generic scan) path honours the halo too."""
    ql = synth.STOCK_STREAM + (" @info(name='query1') from every e1=StockStream[price > 20 and volume > 100] -> "
                               "e2=StockStream[price > e1.price + 5.0] within 500 milliseconds "
                               "select e1.symbol, e2.price insert into Out;")
    _split_run(ql, 50_000, 500, 1, 3, 500, 2)

