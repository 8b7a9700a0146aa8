"""Config 5 as bench.py times it, against the oracle, at bench scale: the whole app (synth.CONFIG5_FULL_QL: an
upstream `#window.time(5 sec)` with sum/group-by inserting into VolStream, and the partitioned logical + absent
pattern over StockStream and VolStream), the round-robin key stream of 1000 keys, per-event playback sends
(every send is one InputHandler.send, advances the clock and fires the Scheduler: InputHandler.java:59-70), and
the default knobs (the compiled NFA kernel for these flushes, the dense tick index, the event prefilter).
2M sends in two pushes of 1M (one flush each, the second continuing every key, window and Scheduler queue from
the first).  Bit for bit: rows, timestamps, callback grouping."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

K = 1000
STOCK_TYPES = ["STRING", "FLOAT", "INT"]


@pytest.fixture(autouse=True)
def _defaults(monkeypatch):
    for k in ("SG_NFA_SPEC", "SG_NFA_TPB", "SG_NFA_RTC", "SG_NFA_RTC_MIN", "SG_NFA_TICK_SEARCH", "SG_NFA_NO_LDS"):
        monkeypatch.delenv(k, raising=False)


@pytest.mark.parametrize("host_chain", [False, True])
def test_config5_bench_size_matches_oracle(host_chain, monkeypatch):
    """host_chain False: the window's output rows stay in HBM into the NFA event store (the default, DevChain in
    api.hip dispatch); True: SG_HOST_CHAIN=1, the rows cross to the host and back as a host push."""
    if host_chain:
        monkeypatch.setenv("SG_HOST_CHAIN", "1")
    n, half = 2_000_000, 1_000_000
    d = synth.stock_ticks_rr(n, synth.SEEDS[5], K)
    g = GpuApp(synth.CONFIG5_FULL_QL)
    g.add_query_callback("query1")
    g.start()
    ids = intern_symbols(g, K)
    assert g.path("query1") == "nfa" and g.path("window") == "window_agg"
    sym = ids[d["symbol"]].astype(np.int32)
    parts, stats = [], []
    for lo in (0, half):
        sl = slice(lo, lo + half)
        g.send_columns("StockStream", d["ts"][sl], [sym[sl], d["price"][sl], d["volume"][sl]], False)   # per-event
        parts.append(g.raw_outputs())
        stats.append({k: g.kernel_ms(k) for k in ("k_nfa_lanes", "nfa_compiled", "nfa_exact_rounds",
                                                 "nfa_chain_device_rows")})
    print(stats)
    assert all(s["nfa_compiled"] == 1 for s in stats), stats       # the bench's kernel
    assert all(s["nfa_exact_rounds"] <= 0 for s in stats), stats   # the jittered stream shares no deadline
    assert all((s["nfa_chain_device_rows"] == 0) == host_chain for s in stats), stats
    o = OracleApp(synth.CONFIG5_FULL_QL)
    o.add_query_callback("query1")
    o.start()
    assert np.array_equal(intern_symbols(o, K), ids)
    si = o.L.or_stream_index(o.h, b"StockStream")
    raw = raw_matrix(STOCK_TYPES, [sym, d["price"], d["volume"]])
    for lo in (0, half):
        o.send_columns(si, d["ts"][lo:lo + half], raw[lo:lo + half], None, False)
    cb = {f: np.concatenate([p[0][f] for p in parts]) for f in parts[0][0]}
    merged = (cb, np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]),
              np.concatenate([p[3] for p in parts]))
    compare_raw(o.raw_outputs(), merged, 3)
    assert len(merged[1]) > 10_000
