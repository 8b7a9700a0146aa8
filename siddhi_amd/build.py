"""Build libsiddhi_gfx.so (HIP kernels + host runtime + C ABI) for gfx950 with hipcc, in-tree."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libsiddhi_gfx.so")
SOURCES = ["api.hip", "followed_by.hip", "keyed_fb.hip", "nfa.hip", "window_agg.hip", "window_gen.hip"]
HEADERS = sorted(f for f in os.listdir(CSRC) if f.endswith(".hpp"))   # every in-tree header
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
         "-I" + os.path.join(HERE, "..", "include")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    hdr_t = max(hdr_t, _mtime(os.path.join(HERE, "..", "include", "siddhi_gfx.h")))
    objs, jobs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT, s.replace(".hip", ".o"))
        objs.append(obj)
        if force or _mtime(obj) < max(_mtime(src), hdr_t):
            jobs.append([HIPCC] + FLAGS + ["-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stderr[-4000:]}")
        return r

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as pool:
        list(pool.map(run, jobs))
    if jobs or not os.path.exists(LIB):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
