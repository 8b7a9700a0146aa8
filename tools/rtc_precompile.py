"""Compile the NFA kernels of every reference KAT (tests/golden/kats.json) into an RTC code-object cache on the CPU,
so that a GPU run of the full compiled-KAT sweep (tools/gpu_run.sh rtcall) loads them instead of compiling on the box.

    SG_RTC_CACHE=siddhi_amd/_build/rtc_kats python tools/rtc_precompile.py [workers]
    python tools/rtc_precompile.py [workers] --suite     (into the default cache next to the library)

--suite compiles what the default GPU suite and the bench run compiled: the sampled KATs of test_gpu_nfa_rtc.py
(kat.rtc_sample),
the configs 3 and 5, and the apps of test_gpu_nfa_expiry.py, so that no GPU test waits on hipRTC.
hipRTC needs no device (sg_query_compile); the workers are processes, since hipRTC serialises the compiles of one
process."""
import os
import sys
import threading
import time
from concurrent.futures import ProcessPoolExecutor, as_completed

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from siddhi_amd.runtime import GpuApp, SiddhiGfxError  # noqa: E402
from kat import load_kats, rtc_sample  # noqa: E402


def one(kat):
    try:
        g = GpuApp(kat["app"] if isinstance(kat, dict) else kat)
    except SiddhiGfxError:
        return 0
    n = 0
    try:
        for q in g.queries:
            if g.path(q) == "nfa":
                g.compile_kernel(q)
                n += 1
    finally:
        g.close()
    return n


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    workers = int(args[0]) if args else 8
    kats = [k for k in load_kats() if not k["expect"].get("create_error")]
    if "--suite" in sys.argv:
        from siddhi_amd import synth
        import test_gpu_nfa_expiry as ex
        kats = rtc_sample(kats) + [synth.CONFIG3_QL, synth.CONFIG5_FULL_QL] + [
            ex.q(b, p) for b in (ex.LONG_PENDING, ex.BURST_NEW, ex.SEQ_WITHIN) for p in (False, True)]
    t0 = time.time()
    done = 0
    nq = 0
    with ProcessPoolExecutor(max_workers=workers) as ex:   # (processes: hipRTC serialises the threads of one)
        for f in as_completed([ex.submit(one, k) for k in kats]):
            nq += f.result()
            done += 1
            if done % 20 == 0:
                print(f"{done}/{len(kats)} KATs, {nq} NFA queries, {time.time() - t0:.0f} s", flush=True)
    print(f"done: {len(kats)} KATs, {nq} NFA queries, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
