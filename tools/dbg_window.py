"""Print the first differing output rows of a window query (oracle vs device) — debugging aid."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import test_gpu_window as T
from synth_run import feed_both

sel = sys.argv[1] if len(sys.argv) > 1 else "select symbol, min(price) as lo, max(volume) as hv, avg(volume) as av group by symbol"
ql = T.BATCH_QL.format(L=97, sel=sel)
o, g, ids = T._pair(ql, 12)
d = T._stock(20_000, 35, 12, 1)
feed_both(o, g, "StockStream", T.STOCK_TYPES, d["ts"], [ids[d["symbol"]], d["price"], d["volume"]], chunk=1_500,
          flush_each=True)
ocb, ots, oraw, onul = o.raw_outputs()
gcb, gts, graw, gnul = g.raw_outputs()
print("rows", len(ots), len(gts))
bad = np.nonzero((oraw[:, :4] != graw[:, :4]).any(axis=1))[0]
print("bad rows", len(bad))
for r in bad[:8]:
    print(r, ots[r], oraw[r, :4], graw[r, :4], onul[r, :4], gnul[r, :4])
