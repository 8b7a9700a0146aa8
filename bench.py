"""Benchmark of the MI355X Siddhi pattern path on BASELINE.json's metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4|1|2] [--events N_PER_GPU]

Default workload (--config 4): the metric's keyed `every a->b within` pattern, BASELINE config 4:

    partition with (symbol of StockStream) begin
      from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
      select e1.symbol, e2.price insert into Out;
    end;

over synthetic ticks (splitmix64 generator of BASELINE.md / SURVEY §8d, seed 0xC0FF04, K=1M symbols,
E=1000 events/ms), generated on the GPU and resident in HBM before timing.  One step = one pass of
the keyed path over the batch: sg_reset + sg_push_device (zero-copy adopt) + sg_flush_device (key
sort, per-key followed-by scan, (j, i) ordering, select-list projection into HBM output columns).

N > 1 (one process per GPU, torch.distributed over RCCL): every rank owns a contiguous time range of
N_PER_GPU ticks (weak scaling) and the step starts with the real exchange of a keyed query — an
all-to-all that routes each event to the rank owning its key (key % N), source-rank order preserving
per-key arrival order — followed by the keyed path on the events received.  The timed region is
bracketed by barrier + synchronize, and the max over ranks is reported.

--config 1: the unkeyed config-1 pattern (time-tiled LDS kernel), 100M ticks/GPU, K=1000.
--config 2: filter + length(1000) window + group-by avg/sum/count (§8 A13-A15), 100M ticks, per-event
            chunking (every filtered event is an output row, written to HBM).
--config 5: the whole config-5 app (synth.CONFIG5_FULL_QL): a time(5 sec) window with sum/group-by
            feeding a partitioned `every (e1 and e2) -> not VolStream[...] for 5 sec` through an inserted
            stream, @app:playback, per-event sends (K=1000 round-robin keys, 10M ticks), host ingest (the caller's columns in pinned memory).
--config 3: `every e1=S, e2=S[price>e1.price]+, e3=S[price<e2[last].price]` partitioned by symbol
            (K=1000, 10M ticks) on the NFA lanes (nfa.hip): device-resident ingest (sg_push_device: the
            columns are copied device to device; the partition keys come to the host for the instance
            bookkeeping), each key's timeline cut into speculative segments (NfaExec::run_spec) whose
            records are kept once the segment's starting state is verified.

Prints ONE JSON line (rank 0) with the metric, the roofline of the dominant kernel (HIP events on the
stream the kernels run on) and the CPU baseline (oracle/ restatement of siddhi-core on the host's
cores, key-sharded for partitioned configs, on a bounded sample of the same workload).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
METRIC = "input events/sec (node) for keyed `every a->b within` pattern; matches/sec"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", type=int, default=4, choices=[1, 2, 3, 4, 5])
    p.add_argument("--events", type=int, default=None, help="events per GPU")
    p.add_argument("--cpu-sample", type=int, default=None)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the end-to-end ordered-output sample (profiling runs)")
    return p.parse_args()


CFG = {
    4: dict(ql="CONFIG4_QL", seed=4, k=1_000_000, e=1000, events=1_000_000_000, cpu_sample=16_000_000,
            workload="config4: partition with (symbol of StockStream) begin from every e1=StockStream[price>20] -> "
                     "e2=StockStream[price>e1.price] within 1 sec select e1.symbol, e2.price end"),
    1: dict(ql="CONFIG1_QL", seed=1, k=1000, e=1, events=100_000_000, cpu_sample=16_000_000,
            workload="config1: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
                     "select e1.symbol, e2.price"),
    3: dict(ql="CONFIG3_QL", seed=3, k=1000, e=1, events=10_000_000, cpu_sample=10_000_000,
            workload="config3: partition with (symbol of StockStream) begin from every e1=StockStream, "
                     "e2=StockStream[price>e1.price]+, e3=StockStream[price<e2[last].price] select e1.symbol, "
                     "e1.price, e2[last].price, e3.price end (device-resident ingest)"),
    5: dict(ql="CONFIG5_FULL_QL", seed=5, k=1000, e=1, events=10_000_000, cpu_sample=10_000_000, rr=True,
            workload="config5: from StockStream#window.time(5 sec) select symbol, sum(volume) as vol5 group by "
                     "symbol insert into VolStream; partition with (symbol of StockStream, symbol of VolStream) "
                     "begin from every (e1=StockStream[price>80] and e2=StockStream[volume>900]) -> "
                     "not VolStream[vol5>4500] for 5 sec end (@app:playback, per-event sends, round-robin keys: "
                     "jittered deadlines; host ingest from pinned buffers)"),
    2: dict(ql="CONFIG2_QL", seed=2, k=1000, e=1, events=100_000_000, cpu_sample=16_000_000,
            workload="config2: from StockStream[price>20]#window.length(1000) select symbol, avg(price), "
                     "sum(price), count() group by symbol (per-event chunks)"),
}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Host threads for the per-GPU CPU baseline: the box's CPU share (16 per GPU on the pool; os.cpu_count()
    reports the whole machine there)."""
    return max(1, min(16, nproc()))


def nproc():
    """`nproc`: the CPUs this process may run on (its affinity mask)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs' worth of time the container's cgroup grants (cpu.max / cfs quota), None when unlimited.  On the GPU
    pool the affinity mask shows the whole machine while the quota is the box's share: threads beyond the quota
    only time-slice (round 4 measured 256 threads no faster than 16)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def usable_cpus():
    """The CPUs the process can actually run in parallel: its affinity mask capped by the cgroup quota."""
    q = cpu_quota()
    return nproc() if q is None else max(1, min(nproc(), q))


def cpu_baseline(cfg, n_events: int, full=None, threads=None):
    """oracle/ restatement of siddhi-core (C++), timed on the host on a bounded sample.

    Partitioned configs (3, 4, 5) run key-sharded on cpu_threads() threads (oracle.pyoracle.sharded_run,
    bit-identical to one app: tests/test_oracle_sharded.py).  Config 4's sample is every event of the
    timed stream whose key is below a cut-off, so each sampled key keeps the timed stream's density
    (~1 event per key per `within` window, ~1000 events per key); unpartitioned configs 1/2 run one
    thread over the stream's first events."""
    from oracle.pyoracle import OracleApp, sharded_run
    from siddhi_amd import synth
    from tests.synth_run import intern_symbols, raw_matrix
    ql = getattr(synth, cfg["ql"])
    batch = cfg is not CFG[2] and cfg is not CFG[5]
    partitioned = cfg in (CFG[3], CFG[4], CFG[5])
    if cfg is CFG[4] and full is not None:
        ts_t, sym_t, price_t, vol_t, n_full = full
        cut = max(1, min(cfg["k"], int(cfg["k"] * n_events / max(n_full, 1))))
        keep = sym_t < cut
        d = {"ts": ts_t[keep].cpu().numpy(), "symbol": sym_t[keep].cpu().numpy().astype(np.int32),
             "price": price_t[keep].cpu().numpy(), "volume": vol_t[keep].cpu().numpy()}
        what = (f"every event of the timed {n_full}-event stream whose key is one of the first {cut} of "
                f"{cfg['k']} symbols ({len(d['ts'])} events, same per-key density as the timed stream)")
        nk = cut
    else:
        if cfg.get("rr"):
            d = synth.stock_ticks_rr(n_events, seed=synth.SEEDS[cfg["seed"]], k=cfg["k"])
        else:
            d = synth.stock_ticks(n_events, seed=synth.SEEDS[cfg["seed"]], k=cfg["k"], e=cfg["e"])
        what = f"the first {n_events} events of the same stream (same generator and seed)"
        if cfg is CFG[5]:
            what += " (each shard's playback clock advances with its own sends: a throughput sample, not a parity run)"
        nk = min(cfg["k"], int(d["symbol"].max()) + 1)
    n = len(d["ts"])
    if partitioned:
        t = threads or cpu_threads()
        raw = raw_matrix(["STRING", "FLOAT", "INT"], [d["symbol"], d["price"], d["volume"]])
        (cbs, _ts, _raw, _nul), dt = sharded_run(ql, "StockStream", d["ts"], raw, d["symbol"] % t, t,
                                                 batch=batch, symbols=nk, shard_key=d["symbol"])
    else:
        t = 1
        o = OracleApp(ql)
        o.add_query_callback("query1")
        o.start()
        ids = intern_symbols(o, nk)
        si = o.L.or_stream_index(o.h, b"StockStream")
        raw = raw_matrix(["STRING", "FLOAT", "INT"], [ids[d["symbol"]], d["price"], d["volume"]])
        t0 = time.perf_counter()
        o.send_columns(si, d["ts"], raw, None, batch)
        dt = time.perf_counter() - t0
        cbs, _ts, _raw, _nul = o.raw_outputs()
    rows = int(cbs["n_in"].sum())
    return {"value": n / dt, "unit": "events/s", "cores": t, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"{what}; {rows} output rows in {dt:.2f} s on {t} thread(s)"
                      f"{' (key-sharded, merged by arrival index)' if partitioned else ''}; siddhi-core "
                      "semantics restated in C++ (oracle/siddhi_oracle.cpp), not the JVM"}


def route_by_key(dist, world, dev, cols, key, ts_base=None):
    """All-to-all: event -> rank (key % world).  Stable grouping by destination keeps per-key order, and
    source-rank order of the received segments keeps it across ranks (PartitionStreamReceiver routes each
    event to its key's instance, PartitionStreamReceiver.java:82-282).

    The destination is one byte, so the stable grouping is a single 8-bit radix pass; each column's
    all-to-all is issued asynchronously (RCCL's stream) while the next column is gathered.  Only the
    columns the query reads travel (ts, symbol, price), and an int64 timestamp column (cols[0] when
    ts_base is given) travels as a 32-bit offset from ts_base: 12 B/event over xGMI."""
    import torch
    if ts_base is not None:
        cols = [(cols[0] - ts_base).to(torch.int32)] + list(cols[1:])
    dest = (key % world).to(torch.uint8)
    order = torch.sort(dest, stable=True).indices
    send_counts = torch.bincount(dest, minlength=world)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    out, works = [], []
    for c in cols:
        src = c.index_select(0, order)
        dst = torch.empty(sum(rc), dtype=c.dtype, device=dev)
        works.append(dist.all_to_all_single(dst, src, rc, sc, async_op=True))
        out.append(dst)
    for w in works:
        w.wait()
    if ts_base is not None:
        out[0] = out[0].to(torch.int64) + ts_base
    return out


def halo_exchange(dist, rank, world, dev, cols, ts, within):
    """Config 1 split by time: rank g also needs the next rank's leading events within W of
    its range's end.  Every rank sends its events with ts <= ts_first + W (a superset: ts_last(g) <=
    ts_first(g+1)) to rank g-1 with one point-to-point send per column and receives rank g+1's.
    Returns the received halo columns (empty on the last rank)."""
    import torch
    cnt = torch.searchsorted(ts, ts[:1] + within, right=True).to(torch.int64)
    got = torch.zeros(1, dtype=torch.int64, device=dev)
    ops = []
    if rank > 0:
        ops.append(dist.P2POp(dist.isend, cnt, rank - 1))
    if rank + 1 < world:
        ops.append(dist.P2POp(dist.irecv, got, rank + 1))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    nsend, nrecv = int(cnt.item()), int(got.item())
    halo = [torch.empty(nrecv, dtype=c.dtype, device=dev) for c in cols]
    ops = []
    for c, h in zip(cols, halo):
        if rank > 0:
            ops.append(dist.P2POp(dist.isend, c[:nsend].contiguous(), rank - 1))
        if rank + 1 < world and nrecv > 0:
            ops.append(dist.P2POp(dist.irecv, h, rank + 1))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return halo


class HostStagedDist:
    """torch.distributed over gloo with device tensors staged through host memory: the one-GPU rehearsal of the
    N-rank bench (SG_BENCH_DIST=gloo, every rank on cuda:0; gloo has no device collectives).  The collectives the
    routed configs issue (all_to_all_single, all_gather, all_reduce, barrier, object gathers) keep their meaning;
    timings of such a run measure the host staging, not xGMI."""

    class _Done:
        def wait(self):
            return None

    def __init__(self, dist):
        self.d = dist
        self.ReduceOp = dist.ReduceOp

    def __getattr__(self, k):
        return getattr(self.d, k)

    def all_to_all_single(self, out, inp, out_split=None, in_split=None, async_op=False):
        o = out.cpu()
        self.d.all_to_all_single(o, inp.cpu(), out_split, in_split)
        out.copy_(o)
        return self._Done() if async_op else None

    def all_gather(self, outs, t):
        os_ = [o.cpu() for o in outs]
        self.d.all_gather(os_, t.cpu())
        for o, h in zip(outs, os_):
            o.copy_(h)

    def all_reduce(self, t, op=None):
        h = t.cpu()
        self.d.all_reduce(h, op=op if op is not None else self.d.ReduceOp.SUM)
        t.copy_(h)


def main():
    a = parse()
    cfg = CFG[a.config]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("SG_BENCH_DIST") == "gloo"   # one-GPU rehearsal of the N-rank path
    if rehearsal:
        local = 0
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as tdist
        if rehearsal:
            tdist.init_process_group("gloo")
            dist = HostStagedDist(tdist)
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist = tdist

    from siddhi_amd import synth
    from siddhi_amd.runtime import GpuApp

    n = a.events or cfg["events"]
    dev = torch.device("cuda", local)
    ql = getattr(synth, cfg["ql"])
    g = GpuApp(ql, device=local)
    # dictionary ids of "S0".."S{K-1}" are consecutive: id = base + symbol index
    base = g.intern("S0")
    for i in range(1, cfg["k"]):
        g.intern(f"S{i}")
    assert g.intern(f"S{cfg['k'] - 1}") == base + cfg["k"] - 1
    # this rank's contiguous time range of the global stream, generated in HBM
    d = synth.stock_ticks_torch(n, seed=synth.SEEDS[cfg["seed"]], k=cfg["k"], e=cfg["e"], start=rank * n, device=dev)
    if cfg.get("rr"):   # round-robin keys (synth.stock_ticks_rr): every key owns a residue of event time
        d["symbol"] = (torch.arange(rank * n, rank * n + n, device=dev, dtype=torch.int64) % cfg["k"]).to(torch.int32)
    t_ts, t_sym, t_price, t_vol = d["ts"], d["symbol"] + base, d["price"], d["volume"]
    del d
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    routed = world > 1 and a.config in (3, 4, 5)
    haloed = world > 1 and a.config == 1      # time-range split with a W halo from the next rank
    ts_base = None
    if routed:   # the routed timestamps travel as 32-bit offsets from the job's first timestamp
        tb = t_ts[:1].clone()
        dist.all_reduce(tb, op=dist.ReduceOp.MIN)
        ts_base = int(tb.item())
        span = t_ts[-1:].clone() - ts_base
        dist.all_reduce(span, op=dist.ReduceOp.MAX)
        if int(span.item()) >= (1 << 31):
            ts_base = None                     # too wide for 32-bit offsets: route the int64 column
    processed = [n]
    if routed:
        t_pos = torch.arange(n, device=dev, dtype=torch.int32)
        # receive counts per source rank (same every step: the routing depends on the keys only)
        dest = ((t_sym - base) % world).to(torch.int64)
        sc = torch.bincount(dest, minlength=world)
        rc_ = torch.empty_like(sc)
        dist.all_to_all_single(rc_, sc)
        recv_counts = [rc_]
        seq = [None]
    if a.config == 5 and not routed:   # host-ingest path (per-event playback sends drive the Scheduler clock)
        # the caller's host columns in pinned memory, as the boundary's JVM shim hands them over (direct ByteBuffers
        # over page-locked memory): the pushes' copies run at the PCIe rate (SG_BENCH_PAGEABLE=1:
        # ordinary pageable numpy arrays)
        pin = os.environ.get("SG_BENCH_PAGEABLE") != "1"
        h_keep = [t.cpu().pin_memory() if pin else t.cpu() for t in (t_ts, t_sym, t_price, t_vol)]
        h_ts, h_cols = h_keep[0].numpy(), [x.numpy() for x in h_keep[1:]]
    stream_protocol = os.environ.get("SG_SHARD_PROTOCOL", "stream") != "batch"
    resolver = None
    if a.config == 5 and routed:
        from siddhi_amd import shard
        shard.check_dictionaries(dist, g, cfg["k"] + base)
        key_hash = lambda key: shard.java_hash(g.string(int(key)))   # noqa: E731
        # the streaming protocol (shard mode 3): the rank's flushes ask the resolver, which all-gathers the logs
        if stream_protocol:
            resolver = shard.StreamingResolver(dist, g, "query1", key_hash)

    def step5_sharded():
        """Config 5 on `world` ranks: the events travel to their key's owner (RCCL all-to-all), the
        global send timestamps to every rank (all-gather: each global send ticks every rank's Schedulers, as
        InputHandler.send -> setCurrentTimestamp does in the single runtime), each rank pushes its share of the
        global sends (sg_push_shard, per-event playback sends) and the cross-rank Scheduler collision protocol
        settles the run: by default the streaming protocol (shard.StreamingResolver: the flush runs as a single
        runtime and asks the driver -- one all-gather of the logs per question -- whether the run collides and who
        loses in each window of the sweep); SG_SHARD_PROTOCOL=batch: shard.settle_collisions_dist (whole-run
        rounds, a tensor exchange of the firing triples first; the logs travel only when two instances share a
        deadline)."""
        g.reset()
        if resolver is not None:
            resolver.reset()
        tsr, sym, price, vol, pos = route_by_key(dist, world, dev, [t_ts, t_sym, t_price, t_vol, t_pos], t_sym - base,
                                                 ts_base)
        src = torch.repeat_interleave(torch.arange(world, device=dev, dtype=torch.int64), recv_counts[0])
        sq = src * n + pos.to(torch.int64)
        off = (t_ts - ts_base).to(torch.int32) if ts_base is not None else t_ts
        gl = [torch.empty_like(off) for _ in range(world)]
        dist.all_gather(gl, off)
        gts = torch.cat(gl)
        h = [x.cpu().numpy() for x in (tsr, sym, price, vol, sq, gts)]
        h_gts = h[5].astype(np.int64) + (ts_base or 0) if ts_base is not None else h[5]
        g.push_shard("StockStream", h[0], [h[1], h[2], h[3]], h[4], h_gts, 0, batch=False)
        if resolver is not None:
            g.flush_device(hip_stream=stream)
        else:
            shard.settle_collisions_dist(dist, g, "query1", key_hash, device=dev,
                                         collect=lambda: g.flush_device(hip_stream=stream))

    def step():
        if a.config == 5 and routed:
            step5_sharded()
            return
        if a.config == 5:
            g.reset()
            g.send_columns("StockStream", h_ts, h_cols, False)   # per-event sends
            g.flush_device(hip_stream=stream)
            return
        ts, sym, price = t_ts, t_sym, t_price
        vol_ptr = t_vol.data_ptr()
        seq_ptr = 0
        if routed:
            # volume is not referenced by the config-4 query: it is not routed (NULL column, never read).
            # Each event travels with its 4-B position in its source range; the source rank is implicit
            # (segments arrive in source-rank order), so the global arrival index is rebuilt on arrival
            # and handed to the runtime for the ordered merge of the ranks' outputs (siddhi_amd/shard.py)
            ts, sym, price, pos = route_by_key(dist, world, dev, [t_ts, t_sym, t_price, t_pos], t_sym - base, ts_base)
            src = torch.repeat_interleave(torch.arange(world, device=dev, dtype=torch.int64), recv_counts[0])
            seq[0] = src * n + pos.to(torch.int64)
            seq_ptr = seq[0].data_ptr()
            vol_ptr = 0                      # (configs 3 and 4 do not read volume)
        n_halo = 0
        if haloed:
            halo = halo_exchange(dist, rank, world, dev, [t_ts, t_sym, t_price], t_ts, 1000)   # within 1 sec
            n_halo = halo[0].numel()
            if n_halo:
                ts, sym, price = (torch.cat([c, h]) for c, h in zip([t_ts, t_sym, t_price], halo))
                vol_ptr = 0        # volume is not referenced by the config-1 query
        g.reset()
        g.push_device("StockStream", ts.numel(), ts.data_ptr(), [sym.data_ptr(), price.data_ptr(), vol_ptr],
                      hip_stream=stream, batch=a.config != 2, seq_ptr=seq_ptr)
        if n_halo:
            g.set_halo("StockStream", n_halo)
        g.flush_device(hip_stream=stream)
        processed[0] = ts.numel() - n_halo

    if a.config in (3, 5):
        # the NFA query's kernel is compiled per query (hipRTC, 10-70 s, cached on disk); a streaming caller gets it
        # from a background compile while the interpreter serves, the bench compiles it before the warm-up so that
        # every timed step runs it
        g.compile_kernel("query1")
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    step_t = []
    for _ in range(a.steps):
        ts0 = time.perf_counter()
        step()
        if os.environ.get("SG_KT_DEBUG"):
            torch.cuda.synchronize()
            step_t.append((time.perf_counter() - ts0) * 1e3)
        kms.append({k: g.kernel_ms(k) for k in KERNELS[a.config]})
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if step_t:
        print("[bench] step ms", [round(x, 2) for x in step_t], file=sys.stderr)
    m = g.match_count("query1")
    e2e_routed = [None]
    if routed and a.config in (3, 4) and not a.no_e2e:
        # the routed step with its match outputs gathered back to the host and merged into single-runtime order
        # (outside the timed region, on a sample of every rank's range): north_star's "gathered back to the host"
        e2e_routed[0] = routed_end_to_end(dist, world, rank, dev, ql, cfg, n, base, t_ts, t_sym, t_price, ts_base,
                                          4_000_000 if a.config == 4 else 2_000_000)
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
        step_s = dt / a.steps
        kmean = {k: float(np.mean([x[k] for x in kms])) for k in KERNELS[a.config]}
        roof = roofline(a.config, processed[0], m, kmean)   # rank 0's own events and matches
        line = {
            "metric": METRIC,
            "value": n * world / step_s,
            "unit": "events/s",
            "matches_per_s": m_total / step_s,
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (splitmix64 ticks per BASELINE.md, generated and resident in HBM)",
            "config": {"workload": cfg["workload"], "events_per_gpu": n, "symbols": cfg["k"],
                       "events_per_ms": cfg["e"], "matches_per_step": m_total,
                       "parallelism": (f"key-hash x{world} (RCCL all-to-all routing, global send clock all-gathered, "
                                       f"{'streaming' if stream_protocol else 'batch'} Scheduler collision protocol)"
                                       if routed and a.config == 5
                                       else f"key-hash x{world} (RCCL all-to-all routing)" if routed
                                       else f"time-range x{world} (W halo from the next rank)" if haloed
                                       else f"time-range x{world}")},
            "roofline": roof,
            "kernel_ms": kmean,
        }
        if rehearsal and world > 1:
            line["rehearsal"] = "all ranks on one GPU, collectives over gloo staged through host memory (not xGMI)"
        if a.config == 4 and world == 1 and not a.no_e2e:
            line["end_to_end"] = end_to_end_sample(t_ts, t_sym, t_price, t_vol, stream, 20_000_000)
        if a.config == 5 and world == 1 and not a.no_e2e:
            line["end_to_end"] = end_to_end_config5(h_ts, h_cols, cfg["k"])
        if e2e_routed[0] is not None:
            line["end_to_end"] = e2e_routed[0]
        if not a.no_cpu and world == 1:
            full = (t_ts, t_sym - base, t_price, t_vol, n) if a.config == 4 else None
            line["cpu_baseline"] = cpu_baseline(cfg, a.cpu_sample or cfg["cpu_sample"], full)
            line["cpu_baseline"]["share"] = "the per-GPU CPU share of the box (16 threads per GPU)"
            line["cpu_baseline"]["cpus"] = {"affinity": nproc(), "cgroup_quota": cpu_quota(), "usable": usable_cpus()}
            if a.config in (3, 4, 5) and usable_cpus() > cpu_threads():
                # the same sample key-sharded over every CPU the process can run in parallel (affinity mask capped
                # by the cgroup quota: threads past the quota only time-slice)
                nb = cpu_baseline(cfg, a.cpu_sample or cfg["cpu_sample"], full, threads=usable_cpus())
                nb["share"] = "every CPU the process can use in parallel (affinity capped by the cgroup quota)"
                line["cpu_baseline_nproc"] = nb
                if nb["value"] < line["cpu_baseline"]["value"]:
                    nb["note"] = (f"slower than {cpu_threads()} threads: the box does not run {nb['cores']} threads "
                                  f"in parallel; the best measured CPU figure is cpu_baseline")
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def end_to_end_sample(ts, sym, price, vol, stream, s):
    """Config 4 with reference-ordered output, on the first `s` events of the resident stream (outside the
    timed region): device pipeline + D2H of the decoded rows and callback boundaries + their copy into the
    caller's arrays (raw_outputs).  Run twice on one runtime (sg_reset between): `cold` includes the first
    allocations of its device and pinned buffers, the second pass is the steady state a streaming runtime
    sees.  Not `value`: that is the device-resident match computation."""
    import torch
    from siddhi_amd import synth
    from siddhi_amd.runtime import GpuApp
    s = min(s, ts.numel())
    try:
        g = GpuApp(synth.CONFIG4_QL, device=torch.cuda.current_device())
        g.add_query_callback("query1")
        g.start()
        res = {}
        for rnd in ("cold", "warm"):
            if rnd == "warm":
                g.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.push_device("StockStream", s, ts.data_ptr(), [sym.data_ptr(), price.data_ptr(), vol.data_ptr()],
                          hip_stream=stream, batch=True)
            g.flush()
            t1 = time.perf_counter()
            cbs, ots, raw, nul = g.raw_outputs(reuse=True)   # drain arrays kept, as the JNI drain's buffers
            t2 = time.perf_counter()
            res[rnd] = (t2 - t0, t1 - t0, t2 - t1, int(len(cbs["kind"])), int(len(ots)))
        dt, tf, to, ncb, nrows = res["warm"]
        return {"events": s, "ms": dt * 1e3, "events_per_s": s / dt, "callbacks": ncb, "rows": nrows,
                "flush_ms": tf * 1e3, "outputs_ms": to * 1e3, "cold_ms": res["cold"][0] * 1e3,
                "includes": "device pipeline, D2H of rows and callback boundaries (flush), copy into the "
                            "caller's numpy arrays (raw_outputs); second pass on one runtime"}
    except Exception as e:   # reported, never fatal to the bench line
        return {"events": s, "error": str(e)[:300]}


def routed_end_to_end(dist, world, rank, dev, ql, cfg, n, base, t_ts, t_sym, t_price, ts_base, s):
    """N > 1, configs 3/4: route the first `s` events of every rank's range to their key owners (RCCL all-to-all),
    run the keyed path with outputs to the host (sg_flush: rows and callback seqs D2H into pinned blocks, then the
    caller's arrays), gather every rank's outputs on rank 0 and merge them by global arrival index into the single
    runtime's callback order (shard.gather_merge, PartitionStreamReceiver's order).  Times are the max over ranks;
    measured outside the timed region, so `value` stays the device-resident step."""
    import torch
    from siddhi_amd import shard
    from siddhi_amd.runtime import GpuApp
    s = min(s, n)
    try:
        g2 = GpuApp(ql, device=torch.cuda.current_device())
        g2.add_query_callback("query1")
        g2.start()
        for i in range(cfg["k"]):
            g2.intern(f"S{i}")
        pos0 = torch.arange(s, device=dev, dtype=torch.int32)
        ph = {}

        def mark(name, t0):
            torch.cuda.synchronize()
            ph[name] = (time.perf_counter() - t0) * 1e3
            return time.perf_counter()
        dist.barrier()
        torch.cuda.synchronize()
        t_start = t = time.perf_counter()
        sym_s = t_sym[:s]
        ts, sym, price, pos = route_by_key(dist, world, dev, [t_ts[:s], sym_s, t_price[:s], pos0], sym_s - base, ts_base)
        sc = torch.bincount(((sym_s - base) % world).to(torch.int64), minlength=world)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc)
        src = torch.repeat_interleave(torch.arange(world, device=dev, dtype=torch.int64), rc)
        seq = src * n + pos.to(torch.int64)            # the global arrival index of the timed stream
        t = mark("route_ms", t)
        g2.push_device("StockStream", ts.numel(), ts.data_ptr(), [sym.data_ptr(), price.data_ptr(), 0],
                       hip_stream=torch.cuda.current_stream(dev).cuda_stream, batch=True, seq_ptr=seq.data_ptr())
        g2.flush()
        t = mark("flush_ms", t)
        part = g2.raw_outputs()
        t = mark("outputs_ms", t)
        merged = shard.gather_merge(dist, part)
        t = mark("gather_merge_ms", t)
        total = (t - t_start) * 1e3
        vals = torch.tensor([ph["route_ms"], ph["flush_ms"], ph["outputs_ms"], ph["gather_merge_ms"], total],
                            dtype=torch.float64, device=dev)
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        v = vals.tolist()
        res = {"events": s * world, "route_ms": v[0], "flush_ms": v[1], "outputs_ms": v[2], "gather_ms": v[3],
               "ms": v[4], "events_per_s": s * world / (v[4] * 1e-3),
               "includes": "RCCL routing, keyed path with outputs D2H to each rank's host (pinned), per-rank decode, "
                           "object gather to rank 0 and the merge by global arrival index (single-runtime order); "
                           "max over ranks per phase"}
        if rank == 0:
            res["rows"] = int(len(merged[1]))
            res["callbacks"] = int(len(merged[0]["kind"]))
        g2.close()
        return res
    except Exception as e:   # reported, never fatal to the bench line
        return {"events": s * world, "error": str(e)[:300]}


def end_to_end_config5(h_ts, h_cols, k):
    """Config 5 with its callbacks delivered (outside the timed region): the same per-event sends, then sg_flush and
    the outputs in the caller's arrays (raw_outputs), second pass on one runtime."""
    from siddhi_amd import synth
    from siddhi_amd.runtime import GpuApp
    try:
        g = GpuApp(synth.CONFIG5_FULL_QL)
        g.add_query_callback("query1")
        g.start()
        for i in range(k):
            g.intern(f"S{i}")
        res = {}
        for rnd in ("cold", "warm"):
            if rnd == "warm":
                g.reset()
            t0 = time.perf_counter()
            g.send_columns("StockStream", h_ts, h_cols, False)
            g.flush()
            t1 = time.perf_counter()
            cbs, ots, raw, nul = g.raw_outputs(reuse=True)
            t2 = time.perf_counter()
            res[rnd] = (t2 - t0, t1 - t0, t2 - t1, int(len(cbs["kind"])), int(len(ots)))
        g.close()
        dt, tf, to, ncb, nrows = res["warm"]
        n = len(h_ts)
        return {"events": n, "ms": dt * 1e3, "events_per_s": n / dt, "callbacks": ncb, "rows": nrows,
                "sends_and_flush_ms": tf * 1e3, "outputs_ms": to * 1e3, "cold_ms": res["cold"][0] * 1e3,
                "includes": "per-event host sends (window query + chained NFA), sg_flush with callbacks in reference "
                            "order, copy into the caller's numpy arrays; second pass on one runtime"}
    except Exception as e:   # reported, never fatal to the bench line
        return {"events": len(h_ts), "error": str(e)[:300]}


KERNELS = {
    4: ["k_kc_sort", "k_kc_slices", "k_kc_match", "k_kt_hist", "k_kt_scatter", "k_kt_match", "k_kt_order", "k_kf_entries",
        "radix_sort", "k_kf_scan", "k_kf_place_order", "total"],
    1: ["k_fb_tile", "k_fb_list_atom"],
    2: ["k_wa_filter_select", "k_wa_gather", "k_wa_tile", "total"],
    3: ["k_nfa_lanes", "k_nfa_spec", "k_nfa_fixup", "nfa_spec_tasks", "nfa_spec_rerun_tasks", "nfa_spec_repaired_tasks",
        "nfa_spec_repair_rounds", "nfa_compiled", "nfa_wide"],
    5: ["k_nfa_lanes", "k_nfa_spec", "k_nfa_fixup", "nfa_spec_tasks", "nfa_spec_rerun_tasks", "nfa_spec_repaired_tasks",
        "nfa_spec_repair_rounds", "nfa_spec_overflows", "nfa_spec_canon_unfit", "nfa_spec_canon_max", "nfa_spec_mismatch",
        "nfa_compiled", "nfa_wide"],
}


def roofline(config, n, m, kms):
    """Dominant kernel's algorithmic bytes / its measured duration."""
    if config == 1:
        # k_fb_tile: per event ts(8)+price(4) read once; per match e1.symbol(4) gathered + {j, symbol, price}(12) written
        k, ms, alg = "k_fb_tile", kms["k_fb_tile"], n * 12 + m * 16
    elif config == 2:
        # whole window pipeline, SURVEY §8d: per event ts(8)+sym(4)+price(4) read + the expired-index re-read (4),
        # per output sym(4)+avg(8)+sum(8)+count(8) written
        k, ms, alg = "window pipeline", kms["total"], n * 20 + m * 28
    elif config in (3, 5):
        # NFA lanes (SURVEY §8d NFA advance): N*(ts 8 + price 4 + sym 4) + M*16 over the lane kernel
        k, ms, alg = "k_nfa_lanes", kms["k_nfa_lanes"], n * 16 + m * 16
    else:
        # keyed pipeline (SURVEY §8d NFA advance): N*(ts 8 + price 4 + sym 4) + M*16
        k, ms, alg = "keyed pipeline", kms["total"], n * 16 + m * 16
    ach = alg / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    traffic, src = pmc_traffic(config, n)
    return {"bound": "hbm", "kernel": k, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src, "kernel_ms": ms,
            "algorithmic_bytes": alg}


def pmc_traffic(config, n):
    """HBM bytes per step of the same workload and the file they come from: the newest committed PMC summary
    (profiles/r*_traffic.json, written by tools/pmc_traffic.py from FETCH_SIZE / WRITE_SIZE passes of this
    bench command, scaled per access width by the calibration run of the same session), or (None, None).
    A bench run cannot profile itself, so the counters come from that named run, not from this one."""
    import glob
    best = (None, None)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == config and d.get("events") == n:
            best = (d["traffic_bytes_per_step"], os.path.relpath(f, ROOT))
    return best


if __name__ == "__main__":
    main()
