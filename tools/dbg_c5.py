import sys, time
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import numpy as np
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import intern_symbols
for n in [100_000, 300_000, 1_000_000, 3_000_000]:
    g = GpuApp(synth.CONFIG5_FULL_QL); g.add_query_callback("query1"); g.start()
    gi = intern_symbols(g, 1000)
    d = synth.stock_ticks_rr(n, synth.SEEDS[5], 1000)
    t = time.time()
    try:
        g.send_columns("StockStream", d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], False)
        g.flush_device()
        print(n, "ok", g.match_count("query1"), round(time.time()-t, 2), g.kernel_ms("k_nfa_lanes"), flush=True)
    except Exception as e:
        print(n, "ERR", e, flush=True)
