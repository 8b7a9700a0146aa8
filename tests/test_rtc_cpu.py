"""CPU-side checks of the run-time compiled NFA kernels (siddhi_amd/csrc/nfa_rtc.hpp), no GPU calls: the
generated source of BASELINE config 3's query carries its lowered table as compile-time constants and its filters
as generated functions, hipRTC compiles it for gfx950 (sg_query_compile needs no device), the code object lands in
the cache, and the kernel keeps its lane state in registers (no private segment: 0 B of scratch) -- config 5's
with the per-processor counters in registers too, config 3's with them in the pools (the generator's fallback when
the compiler would index them dynamically)."""
import glob
import os
import re
import subprocess

import pytest

from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp, SiddhiGfxError

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def test_kernel_source_is_specialised_to_the_table():
    g = GpuApp(synth.CONFIG3_QL)
    src = g.kernel_source("query1")
    # the table: three processors (e1 stream, e2 count <1:-1>, e3 stream), a sequence, constants not loads
    assert "static constexpr int32_t nproc = 3, nslots = 3, seq = 1" in src
    assert "constexpr NProc operator[](int i) const { switch (i) {" in src and "static constexpr A_p p{};" in src
    # filters and projections as generated typed functions (FLOAT compares: cmp(op, T_FLOAT=3, ...))
    assert "sg_prog1(" in src and ", 3, r[" in src
    assert "run_pred" not in src and "Prog* p3" not in src
    assert 'extern "C" __global__' in src and "k_nfa_rtc" in src
    g.close()


def test_no_compiled_kernel_off_the_nfa_path():
    g = GpuApp(synth.CONFIG1_QL)                    # the unkeyed followed-by scan path
    assert g.path("query1") == "followed_by"
    with pytest.raises(SiddhiGfxError) as e:
        g.kernel_source("query1")
    assert e.value.code == -2
    g.close()


@pytest.mark.parametrize("ql", ["CONFIG3_QL", "CONFIG5_FULL_QL"])
def test_kernel_compiles_without_a_frame(tmp_path, monkeypatch, ql):
    """The compiled lane keeps its state in registers: no frame in scratch (the interpreter's was 700-880 B).  At
    two waves per SIMD (amdgpu_waves_per_eu(2), registers capped at 256: nfa_rtc.hpp) config 5's table spills a few
    registers -- 8 VGPRs, 36 B per lane -- which measured 8.3 ms against 12.7 ms uncapped."""
    monkeypatch.setenv("SG_RTC_CACHE", str(tmp_path))
    g = GpuApp(getattr(synth, ql))
    ms, cached = g.compile_kernel("query1")
    assert not cached and ms > 0
    ms2, cached2 = g.compile_kernel("query1")      # the disk cache serves the second request
    assert cached2 and ms2 == 0
    g.close()
    objs = glob.glob(os.path.join(str(tmp_path), "nfa_*.hsaco"))
    assert len(objs) == 1
    notes = subprocess.run([READELF, "--notes", objs[0]], capture_output=True, text=True, check=True).stdout
    assert ".name:           k_nfa_rtc" in notes
    scratch = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", notes).group(1))
    spills = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", notes).group(1))
    assert scratch <= 64 and spills <= 16, (scratch, spills)
    assert int(re.search(r"\.vgpr_count:\s+(\d+)", notes).group(1)) <= 256      # two waves per SIMD
