"""Host-side time split of the config-5 chain (SG_HOST_TIMING)."""
import os, sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
os.environ["SG_HOST_TIMING"] = "1"
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import intern_symbols
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
g = GpuApp(synth.CONFIG5_FULL_QL); g.add_query_callback("query1"); g.start()
gi = intern_symbols(g, 1000)
d = synth.stock_ticks_rr(n, synth.SEEDS[5], 1000)
t = time.time(); g.send_columns("StockStream", d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], False); t1 = time.time()
g.flush_device(); t2 = time.time()
print(f"push {t1-t:.2f} s flush {t2-t1:.2f} s matches {g.match_count('query1')}", file=sys.stderr)
