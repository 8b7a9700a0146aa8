"""Benchmark: input events/s for `every e1=StockStream[price>20] -> e2=StockStream[price>e1.price]
within 1 sec select e1.symbol, e2.price` (BASELINE.json configs[0] query) on the MI355X path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--events N_EVENTS]

A step = one pass of the pattern path over one batch of N_EVENTS synthetic ticks that are already
resident in HBM (splitmix64 generator of BASELINE.md, seed 0xC0FF01, K=1000 symbols, 1 event/ms):
sg_reset + sg_push_device (zero-copy adopt) + sg_flush_device (match scan, (j,i) ordering,
select-list projection into HBM output columns).  N>1: one process per GPU, each rank processes its
own N_EVENTS-tick time range (weak scaling); see DESIGN.md §Multi-GPU.

Prints ONE JSON line (rank 0) with the BASELINE metric, the roofline of the dominant kernel
(HIP-event timing on the kernel's own stream) and the CPU baseline (the oracle/ restatement timed on
a bounded sample on this host, 1 core).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--events", type=int, default=100_000_000)
    p.add_argument("--cpu-sample", type=int, default=3_000_000)
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def cpu_baseline(n_events: int):
    """oracle/ restatement (siddhi-core semantics in C++, 1 thread) on a bounded sample."""
    from oracle.pyoracle import OracleApp
    from siddhi_amd import synth
    from tests.synth_run import intern_symbols, oracle_feed
    d = synth.stock_ticks(n_events, seed=synth.SEEDS[1], k=1000, e=1)
    o = OracleApp(synth.CONFIG1_QL)
    o.add_query_callback("query1")
    o.start()
    ids = intern_symbols(o, 1000)
    t0 = time.perf_counter()
    oracle_feed(o, "StockStream", d, ids)
    dt = time.perf_counter() - t0
    cbs, _ts, _raw, _nul = o.raw_outputs()
    matches = int(cbs["n_in"].sum())
    return {"value": n_events / dt, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"{n_events} ticks of config 1 (seed 0xC0FF01, K=1000, E=1), "
                      f"{matches} matches in {dt:.2f} s; siddhi-core semantics restated in C++ "
                      "(oracle/siddhi_oracle.cpp), not the JVM"}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from siddhi_amd import synth
    from siddhi_amd.runtime import GpuApp

    n = a.events
    # this rank's time range of the global synthetic stream (weak scaling: n ticks per rank)
    d = synth.stock_ticks(n, seed=synth.SEEDS[1], k=1000, e=1, start=rank * n)
    g = GpuApp(synth.CONFIG1_QL, device=local)
    ids = np.array([g.intern(f"S{i}") for i in range(1000)], np.int32)
    dev = torch.device("cuda", local)
    t_ts = torch.from_numpy(d["ts"]).to(dev)
    t_sym = torch.from_numpy(ids[d["symbol"]]).to(dev)
    t_price = torch.from_numpy(d["price"]).to(dev)
    t_vol = torch.from_numpy(d["volume"]).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        g.reset()
        g.push_device("StockStream", n, t_ts.data_ptr(), [t_sym.data_ptr(), t_price.data_ptr(), t_vol.data_ptr()],
                      hip_stream=stream)
        g.flush_device(hip_stream=stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    for _ in range(a.steps):
        step()
        kms.append(g.kernel_ms("k_fb_tile"))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = g.match_count("query1")
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        mm = torch.tensor([m], dtype=torch.int64, device=dev)
        dist.all_reduce(mm)
        m_total = int(mm.item())
    else:
        m_total = m
    if rank == 0:
        ms_step = dt / a.steps * 1e3
        k_ms = float(np.mean(kms))
        # k_fb_tile algorithmic bytes: per event ts(8)+price(4) read once; per match e1.symbol(4)
        # gathered + {j, symbol, price} (12) written
        alg_bytes = n * 12 + m * 16
        achieved = alg_bytes / (k_ms * 1e-3) / 1e9
        line = {
            "metric": "input events/sec (node) for keyed `every a->b within` pattern; matches/sec",
            "value": n * world / (dt / a.steps),
            "unit": "events/s",
            "matches_per_s": m_total / (dt / a.steps),
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (splitmix64 ticks per BASELINE.md, HBM-resident)",
            "config": {"workload": "config1: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
                                   "within 1 sec select e1.symbol, e2.price",
                       "events_per_gpu": n, "symbols": 1000, "events_per_ms": 1, "matches_per_step": m_total,
                       "parallelism": f"time-range x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_fb_tile", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel_ms": k_ms, "algorithmic_bytes": alg_bytes},
        }
        if not a.no_cpu:
            line["cpu_baseline"] = cpu_baseline(a.cpu_sample)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
