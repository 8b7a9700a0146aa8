"""The run-time compiled NFA kernels (nfa_rtc.hpp: the lane code partially evaluated against one query's lowered
table, filters and projections generated as typed straight-line functions, compiled with hipRTC) against the
oracle, bit for bit, on the shapes of BASELINE configs 3 and 5 and on the reference KATs that lower to the NFA path.
Every test forces the compiled kernel (SG_NFA_RTC=1) and asserts that it ran (kernel_ms "nfa_compiled")."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from kat import check, load_kats, run_app
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
        ran.append(self.kernel_ms("nfa_compiled"))
        return orig(self, *a, **k)

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


def _nfa_kats():
    out = []
    for kat in load_kats():
        if kat["expect"].get("create_error"):
            continue
        try:
            g = GpuApp(kat["app"])
        except SiddhiGfxError:
            continue
        if any(g.path(q) == "nfa" for q in g.queries):
            out.append(kat)
        g.close()
    return out


NFA_KATS = _nfa_kats()
# every KAT when asked (SG_RTC_ALL_KATS=1), else every sixteenth: each distinct table is one hipRTC compile (10-70 s,
# parallel below, then cached on disk)
SAMPLE = NFA_KATS if os.environ.get("SG_RTC_ALL_KATS") else NFA_KATS[::16]


@pytest.fixture(scope="module")
def warm_cache():
    """Compile the sampled KATs' kernels in parallel threads (hipRTC needs no GPU; the GIL is released)."""
    def one(kat):
        g = GpuApp(kat["app"])
        try:
            for q in g.queries:
                if g.path(q) == "nfa":
                    g.compile_kernel(q)
        finally:
            g.close()
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(one, SAMPLE))


@pytest.mark.parametrize("kat", SAMPLE, ids=[k["name"] for k in SAMPLE])
def test_compiled_reference_kat(kat, warm_cache):
    g = GpuApp(kat["app"])
    gout = run_app(g, kat)
    assert check(kat, gout) == []
    oout = run_app(OracleApp(kat["app"]), kat)
    assert gout == oout
    nfa = [q for q in g.queries if g.path(q) == "nfa"]
    assert nfa and g.kernel_ms("nfa_compiled") in (0, 1)
