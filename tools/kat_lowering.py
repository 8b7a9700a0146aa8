"""Which reference KATs the device path lowers (app creation only: runs on a GPU-less host).

    python tools/kat_lowering.py [-v]
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from kat import load_kats  # noqa: E402
from siddhi_amd.runtime import GpuApp, SiddhiGfxError  # noqa: E402


def main():
    ok = 0
    why = collections.Counter()
    kats = load_kats()
    for k in kats:
        try:
            GpuApp(k["app"]).close()
            ok += 1
        except SiddhiGfxError as e:
            msg = str(e).splitlines()[0][:160]
            why[msg] += 1
            if "-v" in sys.argv:
                print(k["name"], msg)
    print(f"lowered {ok} / {len(kats)}")
    for m, c in why.most_common():
        print(f"{c:4}  {m}")


if __name__ == "__main__":
    main()
