"""Run every auto-transcribed KAT (tests/golden/kats_auto.json) through the oracle and report
pass / fail / error per source file.  Review aid for tests/golden/review_kats.py.

    python tools/kat_status.py [substring-filter] [-v]
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from kat import check, load_kats, run_app  # noqa: E402
from oracle.pyoracle import OracleApp  # noqa: E402


def main():
    flt = [a for a in sys.argv[1:] if not a.startswith("-")]
    verbose = "-v" in sys.argv
    stats = collections.defaultdict(collections.Counter)
    for k in load_kats("kats_auto.json"):
        if flt and not any(f in k["name"] for f in flt):
            continue
        f = k["name"].split(".")[0]
        try:
            p = check(k, run_app(OracleApp(k["app"]), k))
            st = "pass" if not p else "FAIL"
            msg = "; ".join(p[:2])
        except Exception as e:  # noqa: BLE001
            st, msg = "ERR", str(e).splitlines()[0][:150]
        stats[f][st] += 1
        if st != "pass" and (verbose or flt):
            print(f"{st:4} {k['name']}: {msg}")
    for f, c in sorted(stats.items()):
        print(f"{f:40} {dict(c)}")


if __name__ == "__main__":
    main()
