"""Debug: the falling-runs stack-matcher case -- first callbacks where the device differs from the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["SG_KS_FORCE"] = "1"
from oracle.pyoracle import OracleApp  # noqa: E402
from siddhi_amd import synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from synth_run import feed_both, intern_symbols  # noqa: E402

n, k = 200_000, 400
d = synth.stock_ticks(n, seed=57, k=k, e=2)
i = np.arange(n)
d["symbol"] = ((i // 20) % k).astype(d["symbol"].dtype)
d["price"] = np.where(i % 20 == 19, np.float32(99.0), np.float32(90.0) - (i % 20).astype(np.float32))
ql = synth.CONFIG4_QL
o = OracleApp(ql); o.add_query_callback("query1"); o.start()
g = GpuApp(ql); g.add_query_callback("query1"); g.start()
ids = intern_symbols(g, k); intern_symbols(o, k)
feed_both(o, g, "StockStream", ["STRING", "FLOAT", "INT"], d["ts"], [ids[d["symbol"]], d["price"], d["volume"]])
oc, ots, oraw, _ = o.raw_outputs()
gc, gts, graw, _ = g.raw_outputs()
print("ks_match", g.kernel_ms("k_ks_match"), "rerun", g.kernel_ms("ks_rerun_tasks"), "reject", g.kernel_ms("ks_reject"))
print("callbacks", len(oc["n_in"]), len(gc["n_in"]), "rows", len(ots), len(gts))
m = min(len(oc["n_in"]), len(gc["n_in"]))
bad = np.nonzero((oc["n_in"][:m] != gc["n_in"][:m]) | (oc["ts"][:m] != gc["ts"][:m]))[0]
print("first differing callbacks", bad[:10])
if len(bad):
    b0 = bad[0]
    for c in range(max(0, b0 - 2), min(m, b0 + 4)):
        print(c, "oracle", oc["ts"][c], oc["n_in"][c], oc["seq"][c] if "seq" in oc else "", "gpu", gc["ts"][c], gc["n_in"][c], gc["seq"][c])
    ro = int(np.sum(oc["n_in"][:b0])); rg = int(np.sum(gc["n_in"][:b0]))
    print("oracle rows", oraw[ro:ro + 25, :2].tolist())
    print("gpu rows", graw[rg:rg + 25, :2].tolist())
