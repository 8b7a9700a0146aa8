"""Build libsiddhi_gfx.so (HIP kernels + host runtime + C ABI) for gfx950 with hipcc, in-tree."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libsiddhi_gfx.so")
SOURCES = ["api.hip", "ext.hip", "followed_by.hip", "keyed_fb.hip", "nfa.hip", "window_agg.hip", "window_gen.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
         "-I" + os.path.join(HERE, "..", "include")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0


def _deps(path, seen=None):
    """The file and every local header it includes, transitively (`#include "..."`)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("#include \""):
                name = line.split("\"")[1]
                for d in (os.path.dirname(path), os.path.join(HERE, "..", "include")):
                    cand = os.path.normpath(os.path.join(d, name))
                    if os.path.exists(cand):
                        _deps(cand, seen)
                        break
    return seen


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    objs, jobs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUT, s.replace(".hip", ".o"))
        objs.append(obj)
        if force or _mtime(obj) < max(_mtime(d) for d in _deps(src)):
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
    if jobs or _mtime(LIB) < max(_mtime(o) for o in objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
