"""Probe: where the config-5 NFA lanes keep their pools (LDS bytes per lane, 0 = HBM) and the kernel time,
on a 200K-event config-5 stream (CONFIG5_FULL_QL), with the pool caps from the environment."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from siddhi_amd import synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from synth_run import gpu_feed, intern_symbols  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
d = synth.stock_ticks_rr(n, synth.SEEDS[5], 1000)
g = GpuApp(synth.CONFIG5_FULL_QL); g.add_query_callback("query1"); g.start()
t0 = time.time()
gpu_feed(g, "StockStream", d, intern_symbols(g, 1000), batch=False)
out = g.raw_outputs()
print(f"n={n} rows={int(np.sum(out[0]['n_in']))} wall={time.time() - t0:.2f}s", {k: g.kernel_ms(k) for k in (
    "k_nfa_lanes", "nfa_lanes_per_wg", "nfa_lane_pool_lds_bytes", "nfa_lane_pool_bytes_needed")}, flush=True)
