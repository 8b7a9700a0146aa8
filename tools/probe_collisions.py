"""Probe: the config-5 pattern shape (logical `and` -> absent for 40 ms, partitioned) on a stream with natural
deadline collisions (random keys, E events per ms, no jitter): exact-replay rounds, wall time, parity vs the
oracle.  usage: python tools/probe_collisions.py N [K] [E]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle.pyoracle import OracleApp  # noqa: E402
from siddhi_amd import synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from synth_run import compare_raw, feed_both, intern_symbols  # noqa: E402
from test_gpu_partitioned_absent import SHARED_AND as ABSENT_AFTER_AND, STOCK_TYPES  # noqa: E402

n = int(sys.argv[1]); k = int(sys.argv[2]) if len(sys.argv) > 2 else 1000; e = int(sys.argv[3]) if len(sys.argv) > 3 else 10
d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 11, k=k, e=e)
o = OracleApp(ABSENT_AFTER_AND); o.add_query_callback("query1"); o.start()
g = GpuApp(ABSENT_AFTER_AND); g.add_query_callback("query1"); g.start()
oi, gi = intern_symbols(o, k), intern_symbols(g, k)
t0 = time.time()
feed_both(o, g, "StockStream", STOCK_TYPES, d["ts"], [gi[d["symbol"]], d["price"], d["volume"]], batch=False)
oo = o.raw_outputs()
t1 = time.time()
go = g.raw_outputs()
t2 = time.time()
compare_raw(oo, go, 3)
print(f"n={n} k={k} e={e}: rows={int(np.sum(go[0]['n_in']))} rounds={g.kernel_ms('nfa_exact_rounds')} "
      f"window runs={g.kernel_ms('nfa_sweep_runs')} "
      f"k_nfa_lanes(last)={g.kernel_ms('k_nfa_lanes'):.1f} ms run={g.kernel_ms('nfa_replay_run_ms'):.0f} ms "
      f"resolve={g.kernel_ms('nfa_replay_resolve_ms'):.0f} ms oracle+feed={t1 - t0:.1f} s gpu flush={t2 - t1:.1f} s  bit-exact", flush=True)
