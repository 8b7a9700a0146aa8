"""Record the cross-rank Scheduler collision protocol of one fixture (GPU box): every protocol round's
per-rank firing / notifyAt logs and the deferrals it applied, for the CPU gloo test of the exchange
(tests/test_shard_collision_cpu.py).  Usage: python tools/record_sched_logs.py [out.npz]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

from siddhi_amd import shard, synth  # noqa: E402
from siddhi_amd.runtime import GpuApp  # noqa: E402
from test_gpu_partitioned_absent import SHARED_AND  # noqa: E402

WORLD, K, E, N = 2, 16, 4, 1600


class Rec:
    """Proxy of a rank app that records what the protocol reads and the deferrals it makes."""
    def __init__(self, app, log, rank):
        self.app, self.log, self.rank = app, log, rank

    def shard_mode(self, q, m):
        self.app.shard_mode(q, m)

    def raw_outputs(self):
        out = self.app.raw_outputs()
        if self.rank == 0:
            self.log.append({"fires": [None] * WORLD, "ops": [None] * WORLD, "defer": []})
        self.log[-1]["n_out"] = self.log[-1].get("n_out", 0) + len(out[0]["kind"])
        return out

    def sched_fires(self, q):
        f = self.app.sched_fires(q)
        self.log[-1]["fires"][self.rank] = f
        return f

    def sched_ops(self, q):
        o = self.app.sched_ops(q)
        self.log[-1]["ops"][self.rank] = o
        return o

    def sched_defer(self, q, key, tick, sched):
        self.log[-1]["defer"].append((self.rank, key, tick, sched))
        self.app.sched_defer(q, key, tick, sched)


def main(path):
    d = synth.stock_ticks(N, seed=synth.SEEDS[5] + 7, k=K, e=E)
    apps, log = [], []
    key = None
    for r in range(WORLD):
        g = GpuApp(SHARED_AND)
        g.add_query_callback("query1")
        g.start()
        ids = np.array([g.intern(f"S{i}") for i in range(K)], np.int32)
        key = ids[d["symbol"]]
        idx = shard.route_host(key, WORLD)[r]
        g.push_shard("StockStream", d["ts"][idx], [key[idx], d["price"][idx], d["volume"][idx]], idx, d["ts"])
        apps.append(g)
    hk = {int(i): shard.java_hash(apps[0].string(int(i))) for i in np.unique(key)}
    shard.settle_collisions([Rec(a, log, r) for r, a in enumerate(apps)], "query1", lambda x: hk[int(x)])
    out = {"world": np.int64(WORLD), "rounds": np.int64(len(log)), "n": np.int64(N), "k": np.int64(K),
           "e": np.int64(E), "key_of_symbol": np.array([apps[0].intern(f"S{i}") for i in range(K)], np.int64),
           "hash_key": np.array(list(hk.keys()), np.int64), "hash_val": np.array(list(hk.values()), np.int64)}
    for i, rd in enumerate(log):
        for r in range(WORLD):
            out[f"fires_{i}_{r}"] = rd["fires"][r]
            if rd["ops"][r] is not None:
                out[f"ops_{i}_{r}"] = rd["ops"][r]
        out[f"defer_{i}"] = np.array(rd["defer"], np.int64).reshape(-1, 4)
    np.savez_compressed(path, **out)
    print(f"{len(log)} protocol rounds, {sum(len(r['defer']) for r in log)} deferrals -> {path}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "tests/golden/sched_collision_w2.npz")
