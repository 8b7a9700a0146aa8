"""The run-time compiled NFA kernels (nfa_rtc.hpp: the lane code partially evaluated against one query's lowered
table, filters and projections generated as typed straight-line functions, compiled with hipRTC) against the
oracle, bit for bit, on the shapes of BASELINE configs 3 and 5 and on the reference KATs that lower to the NFA path.
Every test forces the compiled kernel (SG_NFA_RTC=1) and asserts that it ran (kernel_ms "nfa_compiled")."""
import os
import threading
from concurrent.futures import ThreadPoolExecutor, as_completed

import numpy as np
import pytest

from kat import check, load_kats, rtc_sample, run_app
from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp, SiddhiGfxError

import test_gpu_nfa_bench_defaults as bench_defaults
import test_gpu_partitioned_absent as pabs

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _compiled(monkeypatch):
    monkeypatch.setenv("SG_NFA_RTC", "1")
    for k in ("SG_NFA_SPEC", "SG_NFA_SEG", "SG_NFA_WARM", "SG_NFA_TPB"):
        monkeypatch.delenv(k, raising=False)


def test_compiled_config3_bench_defaults(monkeypatch):
    """Config 3 (count/Kleene sequence, K = 1000) on the bench's device ingest with the default speculative
    segments, compiled: bit-exact vs the oracle."""
    ran = []
    orig = GpuApp.raw_outputs

    def spy(self, *a, **k):
        out = orig(self, *a, **k)               # (raw_outputs flushes: read the flag after it)
        ran.append(self.kernel_ms("nfa_compiled"))
        return out

    monkeypatch.setattr(GpuApp, "raw_outputs", spy)
    bench_defaults.test_config3_bench_defaults_match_oracle()
    assert ran and all(r == 1 for r in ran), ran


def test_compiled_config5_full_app():
    """Config 5 (time window -> partitioned logical + absent pattern with Scheduler ticks), compiled."""
    rows, g = pabs._run(synth.CONFIG5_FULL_QL, pabs.rr_ticks(45_000, synth.SEEDS[5], 1000), 1000, 3, 15_000)
    assert rows > 0
    assert g.kernel_ms("nfa_compiled") == 1


def test_compiled_shared_deadlines_exact_sweep():
    """Instances sharing deadlines: the exact sweep's windows and rounds run the compiled kernel too."""
    d = synth.stock_ticks(1600, seed=synth.SEEDS[5] + 7, k=16, e=4)
    rows, g = pabs._run(pabs.SHARED_AND, d, 16, 3)
    assert rows > 0
    assert g.kernel_ms("nfa_exact_rounds") > 0
    assert g.kernel_ms("nfa_compiled") == 1


KATS = [k for k in load_kats() if not k["expect"].get("create_error")]
# every KAT when asked (SG_RTC_ALL_KATS=1), else kat.rtc_sample: every fortieth and the first two of every test class
# (those on other paths skip).  Each distinct table is one hipRTC compile (10-70 s, cached on disk; the tree ships the
# cache tools/rtc_precompile.py --suite writes).  (No GpuApp at import: the library's HIP runtime must not initialise
# before torch's, conftest.py.)
SAMPLE = KATS if os.environ.get("SG_RTC_ALL_KATS") else rtc_sample(KATS)


def _nfa_queries(g):
    return [q for q in g.queries if g.path(q) == "nfa"]


@pytest.fixture(scope="module")
def warm_cache():
    """Compile the sampled KATs' kernels in parallel threads (hipRTC needs no GPU; the GIL is released)."""
    def one(kat):
        try:
            g = GpuApp(kat["app"])
        except SiddhiGfxError:
            return
        try:
            for q in _nfa_queries(g):
                g.compile_kernel(q)
        finally:
            g.close()
    done = [0]
    stop = threading.Event()

    def beat():                      # progress every 20 s: a silent GPU run is taken as hung
        while not stop.wait(20):
            print(f"compiling: {done[0]}/{len(SAMPLE)} done", flush=True)
    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    try:
        with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
            for f in as_completed([ex.submit(one, k) for k in SAMPLE]):
                f.result()
                done[0] += 1
    finally:
        stop.set()
    print(f"compiled {done[0]}/{len(SAMPLE)}", flush=True)


@pytest.mark.parametrize("kat", SAMPLE, ids=[k["name"] for k in SAMPLE])
def test_compiled_reference_kat(kat, warm_cache):
    try:
        g = GpuApp(kat["app"])
    except SiddhiGfxError as e:
        pytest.skip(f"not lowered: {e}")
    if not _nfa_queries(g):
        pytest.skip("no query on the NFA path")
    gout = run_app(g, kat)
    assert check(kat, gout) == []
    oout = run_app(OracleApp(kat["app"]), kat)
    assert gout == oout
    assert g.kernel_ms("nfa_compiled") in (-1, 1)      # (-1: the KAT never flushed events into an NFA query)


STREAM_QL = (synth.STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') "
             "from every e1=StockStream, e2=StockStream[price > e1.price]+, e3=StockStream[price < e2[last].price] "
             "select e1.symbol, e2[last].price as p2, e3.price as p3 insert into Out; end;")


def test_background_compile_for_a_streaming_caller(monkeypatch, tmp_path):
    """A caller that flushes 4,096-event chunks, with no cached code object (an empty disk cache, a table no other
    test compiles): once the query has run SG_NFA_RTC_MIN events hipRTC compiles its kernel on a background thread
    while the interpreter serves the flushes; no flush waits for the compile; every flush after it is ready runs the
    compiled kernel.  Output bit-exact vs the oracle over the whole run."""
    import time
    from synth_run import compare_raw, intern_symbols, raw_matrix
    monkeypatch.delenv("SG_NFA_RTC", raising=False)          # the default mode (the module fixture forces 1)
    monkeypatch.setenv("SG_RTC_CACHE", str(tmp_path))
    monkeypatch.setenv("SG_NFA_RTC_MIN", "16384")
    o = OracleApp(STREAM_QL); o.add_query_callback("query1"); o.start()
    g = GpuApp(STREAM_QL); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    k, chunk = 100, 4096
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    d = synth.stock_ticks(chunk * 600, seed=synth.SEEDS[3] + 21, k=k, e=2)
    raw = raw_matrix(["STRING", "FLOAT", "INT"], [oi[d["symbol"]], d["price"], d["volume"]])
    si = o.L.or_stream_index(o.h, b"StockStream")
    flags, worst, t_start = [], 0.0, time.time()
    for c in range(600):
        s, e = c * chunk, (c + 1) * chunk
        o.send_columns(si, d["ts"][s:e], raw[s:e], None, True)
        g.send_columns("StockStream", d["ts"][s:e], [gi[d["symbol"][s:e]], d["price"][s:e], d["volume"][s:e]], True)
        t0 = time.time()
        g.flush()
        worst = max(worst, time.time() - t0)
        flags.append(int(g.kernel_ms("nfa_compiled")))
        if flags[-3:] == [1, 1, 1] and len(flags) >= 3:
            break
        if flags[-1] != 1:
            time.sleep(0.25)                                  # (the compile runs on the host meanwhile)
        assert time.time() - t_start < 100, f"no compiled kernel after {len(flags)} flushes"
    first = flags.index(1)
    assert first >= 4, flags                                  # the threshold, then the compile took some flushes
    assert all(f == 0 for f in flags[:first]) and all(f == 1 for f in flags[first:]), flags
    assert g.kernel_ms("nfa_rtc_background") == 1
    assert worst < 5.0, f"a flush took {worst:.1f} s (it waited on hipRTC)"
    compare_raw(o.raw_outputs(), g.raw_outputs(), 3)
    assert any(os.scandir(tmp_path))                          # the compile wrote the disk cache
