"""Debug: deferral sequences of the collision protocol at world 1 vs world 2 (GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from siddhi_amd import shard, synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from test_gpu_partitioned_absent import SHARED_AND  # noqa: E402

K, E, N = 3, 2, 400


class Rec:
    def __init__(self, app, log, rank):
        self.app, self.log, self.rank = app, log, rank

    def shard_mode(self, q, m):
        self.app.shard_mode(q, m)

    def raw_outputs(self):
        return self.app.raw_outputs()

    def sched_fires(self, q):
        return self.app.sched_fires(q)

    def sched_ops(self, q):
        o = self.app.sched_ops(q)
        return o

    def sched_defer(self, q, key, tick, sched):
        self.log.append((key, tick, sched))
        self.app.sched_defer(q, key, tick, sched)


def run(world):
    d = synth.stock_ticks(N, seed=synth.SEEDS[5] + 7, k=K, e=E)
    apps, log = [], []
    for r in range(world):
        g = GpuApp(SHARED_AND)
        g.add_query_callback("query1")
        g.start()
        ids = np.array([g.intern(f"S{i}") for i in range(K)], np.int32)
        key = ids[d["symbol"]]
        idx = shard.route_host(key, world)[r]
        g.push_shard("StockStream", d["ts"][idx], [key[idx], d["price"][idx], d["volume"][idx]], idx, d["ts"])
        apps.append(g)
    hk = lambda x: shard.java_hash(apps[0].string(int(x)))
    recs = [Rec(a, log, r) for r, a in enumerate(apps)]
    # first round logs
    for a in apps:
        a.shard_mode("query1", 2)
    outs = [a.raw_outputs() for a in apps]
    fires = [a.sched_fires("query1") for a in apps]
    ops = [a.sched_ops("query1") for a in apps]
    np.set_printoptions(linewidth=200)
    allf = np.concatenate(fires)
    print(f"world {world}: first collision {shard.first_collision(allf)}; fires {[len(f) for f in fires]} ops {[len(o) for o in ops]}")
    for r in range(world):
        print(" rank", r, "fires[:12]", fires[r][:12].tolist())
        print(" rank", r, "ops[:12]", ops[r][:12].tolist())
    parts = shard.settle_collisions(recs, "query1", hk)
    print(f"world {world}: {len(log)} deferrals: {log[:40]}")
    m = shard.merge_outputs(parts)
    return log, m


l1, m1 = run(1)
l2, m2 = run(2)
for i, (a, b) in enumerate(zip(l1, l2)):
    if a != b:
        print("first deferral difference at", i, a, b)
        break
print("callbacks", len(m1[0]["kind"]), len(m2[0]["kind"]))
c1, c2 = m1[0], m2[0]
for i in range(min(len(c1["seq"]), len(c2["seq"]))):
    if (c1["seq"][i], c1["ts"][i], c1["tsched"][i], c1["tdl"][i]) != (c2["seq"][i], c2["ts"][i], c2["tsched"][i], c2["tdl"][i]):
        print("first callback difference", i, [(c1[f][i], c2[f][i]) for f in ("seq", "ts", "tsched", "tdl", "n_in")])
        break
