"""Probe: protocol rounds of shard.settle_collisions on natural-collision streams (random keys, E events per ms,
the config-5 pattern shape SHARED_AND) at N events over W ranks, bounded by max_rounds.

    python tools/probe_shard_rounds.py N W E [E ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from siddhi_amd import shard, synth  # noqa: E402
from test_gpu_shard_nfa import SHARED_AND, _key_hash, _oracle, _ranks  # noqa: E402
from synth_run import compare_raw  # noqa: E402

n, world = int(sys.argv[1]), int(sys.argv[2])
for e in [int(x) for x in sys.argv[3:]]:
    d = synth.stock_ticks(n, seed=synth.SEEDS[5] + 11, k=1000, e=e)
    ref, ids = _oracle(SHARED_AND, d, 1000)
    apps = _ranks(SHARED_AND, d, 1000, world, ids, clock=True)
    t0 = time.time()
    try:
        parts = shard.settle_collisions(apps, "query1", _key_hash(apps[0]), max_rounds=150)
        compare_raw(ref, shard.merge_outputs(parts), 3)
        print(f"n={n} world={world} e={e}: rounds={shard.last_rounds} {time.time() - t0:.1f} s bit-exact", flush=True)
    except RuntimeError as x:
        print(f"n={n} world={world} e={e}: not settled in 150 rounds ({time.time() - t0:.1f} s): {x}", flush=True)
    for a in apps:
        a.close()
