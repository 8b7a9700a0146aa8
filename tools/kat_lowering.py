"""Which reference KATs lower to which device path (and why the others do not) — run on a GPU box."""
import sys
from collections import Counter
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from kat import load_kats
from siddhi_amd.runtime import GpuApp, SiddhiGfxError

pat = sys.argv[1] if len(sys.argv) > 1 else ""
why, ok = Counter(), Counter()
for k in load_kats():
    src = k.get("source", "") or k.get("name", "")
    if pat not in src:
        continue
    try:
        g = GpuApp(k["app"])
        ok[src.split("::")[0].split(":")[0]] += 1
    except SiddhiGfxError as e:
        why[str(e)[:140]] += 1
print("lowered:", sum(ok.values()), dict(ok))
for w, c in why.most_common(25):
    print(c, w)
