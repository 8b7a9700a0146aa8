"""Config 3 as bench.py times it, against the oracle: device-resident ingest (sg_push_device: the columns copied
device to device, the partition keys to the host for the instance bookkeeping), K = 1000 keys, 1M events per
push, and the DEFAULT speculative-segment settings (no SG_NFA_SPEC / SG_NFA_SEG / SG_NFA_WARM: segments of
128 events with 48-event warm-ups start at 256 events per key and flush, on small scratch pools that double for
the next flush when more than 1 % of the segments overflowed).  Two pushes, each one send(Event[]) of 1M
events (one flush each), so the second flush runs on the pools the first one grew and continues every key
from the state the first one verified.  Bit for bit: rows, timestamps, callback grouping."""
import os

import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

K = 1000


@pytest.fixture(autouse=True)
def _defaults(monkeypatch):
    for k in ("SG_NFA_SPEC", "SG_NFA_SEG", "SG_NFA_WARM", "SG_NFA_TPB"):
        monkeypatch.delenv(k, raising=False)


def test_config3_bench_defaults_match_oracle():
    import torch
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    n, half = 2_000_000, 1_000_000
    d = synth.stock_ticks(n, seed=synth.SEEDS[3], k=K, e=1)
    g = GpuApp(synth.CONFIG3_QL)
    g.add_query_callback("query1")
    g.start()
    ids = intern_symbols(g, K)
    assert g.path("query1") == "nfa"
    sym = ids[d["symbol"]].astype(np.int32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    parts, stats = [], []
    for lo in (0, half):
        ts = torch.from_numpy(d["ts"][lo:lo + half]).to(dev)
        sy = torch.from_numpy(sym[lo:lo + half]).to(dev)
        pr = torch.from_numpy(d["price"][lo:lo + half]).to(dev)
        torch.cuda.synchronize()
        g.push_device("StockStream", half, ts.data_ptr(), [sy.data_ptr(), pr.data_ptr(), 0], hip_stream=stream)
        parts.append(g.raw_outputs())
        stats.append({k: g.kernel_ms(k) for k in ("k_nfa_spec", "nfa_spec_tasks", "nfa_spec_rerun_tasks",
                                                    "nfa_spec_overflows")})
    print(stats)
    assert all(s["k_nfa_spec"] > 0 and s["nfa_spec_tasks"] > 5_000 for s in stats), stats   # segments ran
    o = OracleApp(synth.CONFIG3_QL)
    o.add_query_callback("query1")
    o.start()
    oi = intern_symbols(o, K)
    assert np.array_equal(oi, ids)
    si = o.L.or_stream_index(o.h, b"StockStream")
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [sym, d["price"], np.zeros(n, np.int32)])
    for lo in (0, half):
        o.send_columns(si, d["ts"][lo:lo + half], raw[lo:lo + half], None, True)
    cb = {f: np.concatenate([p[0][f] for p in parts]) for f in parts[0][0]}
    merged = (cb, np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]),
              np.concatenate([p[3] for p in parts]))
    compare_raw(o.raw_outputs(), merged, 4)
    assert len(merged[1]) > 1000
