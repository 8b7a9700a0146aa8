"""Step-by-step smoke with progress on stderr (localises a hang between host and kernel)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
T0 = time.time()


def say(m):
    print(f"[{time.time() - T0:7.2f}s] {m}", file=sys.stderr, flush=True)


say("start")
import numpy as np  # noqa: E402
from siddhi_amd import synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from synth_run import intern_symbols  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
tile = sys.argv[2] if len(sys.argv) > 2 else None
if tile:
    os.environ["SG_FB_TILE_T"], os.environ["SG_FB_TILE_H"] = tile.split(",")
d = synth.stock_ticks(n, seed=synth.SEEDS[1], k=100, e=1)
say("create")
g = GpuApp(synth.CONFIG1_QL, device=0)
say(f"path {g.path('query1')}")
g.add_query_callback("query1")
g.start()
ids = intern_symbols(g, 100)
say("send")
g.send_columns("StockStream", d["ts"], [ids[d["symbol"]], d["price"], d["volume"]], True)
say("flush")
g.flush()
say(f"flushed: {g.match_count('query1')} matches, kernels {g.kernel_ms('k_fb_tile'):.3f} ms")
out = g.raw_outputs()
say(f"outputs {len(out[1])}")
