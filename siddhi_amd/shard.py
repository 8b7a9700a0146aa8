"""Multi-GPU keyed sharding around the C ABI: routing, output gather and the ordered merge.

`partition with (key of S)` instances are independent (PartitionStateHolder keys), so the events of a
key can run on the GPU that owns it: rank = key % world.  Every rank starts with a contiguous time
range of the stream; the all-to-all (bench.route_by_key, RCCL over xGMI) sends each event to its owner
together with its global arrival index, and concatenating the received segments in source-rank order
keeps the arrival order, hence each key's order and non-decreasing timestamps.  Each rank pushes its
events with their global indices (sg_batch.seq), so every callback it produces carries the arrival index
of the send that fired it (sg_out_callback_seq).  A send belongs to one key, hence to one rank: merging
the ranks' callbacks by that index restores the single-runtime callback order of
PartitionStreamReceiver (CORE/partition/PartitionStreamReceiver.java:82-282) exactly.

route_host is the host restatement of the routing (one-GPU rehearsal, tests); gather_merge moves the
outputs to rank 0 over torch.distributed and merges them.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np


def owner(key: np.ndarray, world: int) -> np.ndarray:
    """The rank owning each partition key (bench.route_by_key's destination)."""
    return (np.asarray(key).astype(np.int64) % world).astype(np.int64)


def route_host(key: np.ndarray, world: int) -> List[np.ndarray]:
    """Global indices of the events each rank receives, in the order it receives them.

    Rank r starts with the contiguous range [r*n/world, (r+1)*n/world); the all-to-all concatenates the
    received segments in source-rank order, so each destination's list is increasing."""
    n = len(key)
    dest = owner(key, world)
    bounds = [n * r // world for r in range(world + 1)]
    out = []
    for d in range(world):
        segs = [np.nonzero(dest[bounds[s]:bounds[s + 1]] == d)[0] + bounds[s] for s in range(world)]
        out.append(np.concatenate(segs).astype(np.int64))
    return out


Raw = Tuple[dict, np.ndarray, np.ndarray, np.ndarray]


def merge_outputs(parts: Sequence[Raw]) -> Raw:
    """Merge per-rank raw outputs (GpuApp.raw_outputs: cbs['seq'], and 'tsched' / 'tdl' for callbacks a
    Scheduler tick fired) into single-runtime order: by the arrival seq of the send; at one seq the tick's
    callbacks first (InputHandler.send advances the clock -- firing the Schedulers -- before it dispatches the
    event, InputHandler.java:59-70), those in (scheduler, deadline) order across partition keys (the
    TreeMultimap of Scheduler.onTimeChange, Scheduler.java:74-104); each rank's own order otherwise."""
    parts = [p for p in parts if len(p[0]["kind"])]
    fields = ("kind", "target", "ts", "n_in", "n_rm", "seq", "tsched", "tdl")
    if not parts:
        return ({k: np.zeros(0, np.int64) for k in fields},
                np.zeros(0, np.int64), np.zeros((0, 1), np.int64), np.zeros((0, 1), np.uint8))
    def col(p, f):
        if f in p[0]:
            return p[0][f]
        return np.full(len(p[0]["kind"]), -1 if f == "tsched" else 0, np.int64)
    cat = {f: np.concatenate([col(p, f) for p in parts]) for f in fields}
    phase = np.where(cat["tsched"] >= 0, 0, 1)
    pos = np.arange(len(cat["seq"]))
    order = np.lexsort((pos, cat["tdl"], cat["tsched"], phase, cat["seq"]))
    cbs = {f: cat[f][order] for f in fields}
    nrow = [(p[0]["n_in"] + p[0]["n_rm"]).astype(np.int64) for p in parts]
    base = np.concatenate([[0], np.cumsum([len(p[1]) for p in parts])])
    starts = np.concatenate([base[i] + np.concatenate([[0], np.cumsum(nr)[:-1]]) for i, nr in enumerate(nrow)])[order]
    lens = np.concatenate(nrow)[order]
    tot = int(lens.sum())
    idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(tot)
    width = max(p[2].shape[1] for p in parts)
    raw = np.concatenate([np.pad(p[2], ((0, 0), (0, width - p[2].shape[1]))) for p in parts])[idx]
    nul = np.concatenate([np.pad(p[3], ((0, 0), (0, width - p[3].shape[1])), constant_values=1) for p in parts])[idx]
    ts = np.concatenate([p[1] for p in parts])[idx]
    return cbs, ts, raw, nul


def gather_merge(dist, part: Raw, dst: int = 0):
    """Gather every rank's raw outputs on rank `dst` (torch.distributed object gather) and merge them;
    returns the merged outputs on `dst`, None elsewhere."""
    world = dist.get_world_size()
    box = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(part, box, dst=dst)
    return merge_outputs(box) if dist.get_rank() == dst else None


# --------------------------------------------------------------------------------------------------------
# Cross-rank Scheduler collisions (config 5 sharded by key; include/siddhi_gfx.h sg_query_shard_mode).
#
# Scheduler.notifyAt keeps one SchedulerState per deadline (SchedulerState.compareTo == 0 in the
# TreeMultimap, CORE/util/Scheduler.java:77-97, 120-147), so when instances of several partition keys
# wait on one deadline only the first in the key -> state HashMap's iteration order fires at that tick;
# the others fire at a later tick.  A rank sees its own keys only, so each rank logs its firings (and its
# notifyAt calls) and the resolution below replays the ONE map of the single runtime over the union of the
# logs, in global arrival order, up to the earliest colliding (tick, scheduler); the losers are deferred
# on their owner ranks, which re-run, until no tick collides.  The single-runtime replay in nfa.hip
# (NfaExec::resolve_first_collision) is the same rule over one rank's logs.

def java_hash(s: str) -> int:
    """HashMap.hash(String.hashCode()) as an unsigned 32-bit value (runtime.hpp java_key_hash)."""
    h = 0
    for ch in s.encode():
        h = (31 * h + ch) & 0xFFFFFFFF
    return h ^ (h >> 16)


class JdkHashMap:
    """Iteration order of a java.util.HashMap (JDK 8) under put-if-absent / remove: power-of-two table
    from 16, resize past 0.75 load splitting each bin in order, treeification refused (bins of >= 8
    entries only resize below 64 bins).  Restates nfa.hip NfaExec::SchedMap."""

    def __init__(self):
        self.tab: List[list] = []
        self.size = 0
        self.thr = 0

    def _resize(self):
        old = len(self.tab)
        if old == 0:
            self.tab, self.thr = [[] for _ in range(16)], 12
            return
        nt = [[] for _ in range(old * 2)]
        for b, chain in enumerate(self.tab):
            for h, k in chain:
                nt[b + old if h & old else b].append((h, k))
        self.tab = nt
        self.thr *= 2

    def touch(self, h: int, key: int):
        if self.size > self.thr or not self.tab:
            self._resize()
        chain = self.tab[h & (len(self.tab) - 1)]
        if any(k == key for _h, k in chain):
            return
        cnt = len(chain)
        chain.insert(0, (h, key))
        if cnt >= 7:
            if len(self.tab) < 64:
                self._resize()
            else:
                raise RuntimeError("partition Scheduler map bin would be treeified (not lowered)")
        self.size += 1

    def remove(self, h: int, key: int):
        if not self.tab:
            return
        chain = self.tab[h & (len(self.tab) - 1)]
        for i, (_h, k) in enumerate(chain):
            if k == key:
                del chain[i]
                self.size -= 1
                return

    def rank(self, h: int, key: int):
        if not self.tab:
            return (1 << 62,)
        b = h & (len(self.tab) - 1)
        for i, (_h, k) in enumerate(self.tab[b]):
            if k == key:
                return (b, i)
        return (1 << 62,)


def first_collision(fires: np.ndarray):
    """Earliest (tick, scheduler) at which two instances fired under one head deadline, or None.
    `fires`: the SCHED_FIRE logs of all ranks, concatenated."""
    if len(fires) < 2:
        return None
    o = np.lexsort((fires["head"], fires["sched"], fires["tick"]))
    f = fires[o]
    dup = ((f["tick"][1:] == f["tick"][:-1]) & (f["sched"][1:] == f["sched"][:-1]) &
           (f["head"][1:] == f["head"][:-1]))
    if not dup.any():
        return None
    i = int(np.argmax(dup))
    return int(f["tick"][i]), int(f["sched"][i])


def resolve_collision(fires: Sequence[np.ndarray], ops: Sequence[np.ndarray], key_hash, tick_now=None,
                      min_wait: int = 0) -> list:
    """-> [(rank, key, tick, sched)] to defer, or [] when no tick collides.  fires[r] / ops[r]: rank r's
    SCHED_FIRE / SCHED_OP logs (shard mode 2); key_hash(key) -> java_hash of the key's string.

    The earliest collision's losers always; with the ticks' clocks and the shortest absent wait (sg_query_sched_clock)
    also every later collision the logs still describe exactly, as nfa.hip NfaExec::replay_maps does for one runtime:
    its tick's clock is before the first collision's clock plus the shortest wait (a deferred instance fires late and
    arms its next deadline beyond that), none of its instances was deferred or fired since under a deferral, none of
    its shared heads was deferred, and the map neither resized nor came within the deferred count of its threshold."""
    allf = np.concatenate([np.asarray(f) for f in fires]) if fires else np.zeros(0)
    col = first_collision(allf) if len(allf) else None
    if col is None:
        return []
    ctick, csched = col
    batch = tick_now is not None and min_wait > 0
    if batch:
        clock_end = int(tick_now[ctick]) + int(min_wait)
        last = int(np.searchsorted(np.asarray(tick_now), clock_end, side="left"))   # ticks < last are in reach
        ticks = allf["tick"]
        sel = ticks < last
        cseq = int(allf["seq"][sel].max()) if sel.any() else int(allf["seq"][(ticks == ctick)][0])
    else:
        cseq = int(allf["seq"][(allf["tick"] == ctick)][0])
    # items in single-runtime order: (seq, phase, tick, firing sched, stage, head, event pos, sub)
    # stage 0 = the tick's collection of due states, 1 = notifyAt, 2 = returnAllStates
    items = []
    for r, op in enumerate(ops):
        op = op[op["seq"] <= cseq]
        for o in op.tolist():
            seq, head, key, tick, sub, pos, phase, kfire, ktarget = o[:9]
            if phase == 0:
                items.append((seq, 0, tick, kfire, 1, head, 0, sub, 1, ktarget, key))
            else:
                items.append((seq, 1, -1, -1, 1, 0, pos, sub, 1, ktarget, key))
    fired: dict = {}
    for r, f in enumerate(fires):
        for key, head, seq, tick, sched, empty_after, _p in np.asarray(f).tolist():
            fired.setdefault((tick, sched), []).append((r, key, head, empty_after, seq))
    for (tick, sched), fl in fired.items():
        seq = fl[0][4]
        if seq > cseq:
            continue
        items.append((seq, 0, tick, sched, 0, -(1 << 63), 0, 0, 0, 0, 0))
        items.append((seq, 0, tick, sched, 2, (1 << 63) - 1, 0, 0, 2, 0, 0))
    items.sort(key=lambda t: t[:8])
    maps: dict = {}
    hcache: dict = {}

    def hk(key):
        h = hcache.get(key)
        if h is None:
            h = hcache[key] = key_hash(key)
        return h
    losers: list = []
    first = False
    dkeys: set = set()              # (rank, key) deferred this round
    dheads: set = set()             # (sched, head) they were deferred under
    cap0: dict = {}
    smax: dict = {}
    for it in items:
        kind = it[8]
        if kind == 1:
            m = maps.setdefault(it[9], JdkHashMap())
            m.touch(hk(it[10]), it[10])
            smax[it[9]] = max(smax.get(it[9], 0), m.size)
            continue
        tick, sched = it[2], it[3]
        fl = fired[(tick, sched)]
        m = maps.setdefault(sched, JdkHashMap())
        if kind == 0:
            if first:
                if int(tick_now[tick]) >= clock_end or any((r, key) in dkeys for r, key, _h, _e, _s in fl):
                    return losers
            elif (tick, sched) != (ctick, csched):
                continue
            byhead: dict = {}
            for r, key, head, _e, _s in fl:
                byhead.setdefault(head, []).append((r, key))
            shared = [h for h in sorted(byhead) if len(byhead[h]) >= 2]
            if first and shared:
                if len(m.tab) != cap0.get(sched, 0) or smax.get(sched, 0) + len(dkeys) + 1 > m.thr:
                    return losers
                if any((sched, h) in dheads for h in shared):
                    return losers
            for head in shared:
                grp = byhead[head]
                win = min(grp, key=lambda rk: m.rank(hk(rk[1]), rk[1]))
                for r, key in grp:
                    if (r, key) != win:
                        losers.append((r, key, tick, sched))
                        dkeys.add((r, key))
                        dheads.add((sched, head))
            if not first:
                first = True
                if not batch:
                    return losers
                cap0 = {k: len(v.tab) for k, v in maps.items()}
                smax = {k: v.size for k, v in maps.items()}
            continue
        for r, key, _head, empty_after, _s in fl:   # returnAllStates drops states with empty queues
            if empty_after and (r, key) not in dkeys:
                m.remove(hk(key), key)
    if first:
        return losers
    raise RuntimeError("scheduler replay did not reach the collision")


last_rounds = 0   # diagnostic: protocol rounds of the last settle_collisions(_dist)


def _clock(app, query):
    """(tick clocks, shortest absent wait) of a rank app, or (None, 0): one collision per round then
    (also with SG_SHARD_ONE_PER_ROUND, the comparison hook)."""
    f = getattr(app, "sched_clock", None)
    if f is None or os.environ.get("SG_SHARD_ONE_PER_ROUND"):
        return None, 0
    try:
        return f(query)
    except Exception:
        return None, 0


def settle_collisions(apps: Sequence, query: str, key_hash, max_rounds: int = 100_000) -> List[Raw]:
    """One-process rehearsal of the protocol over the rank apps of one GPU (after every rank pushed its
    share): flush, gather the firing logs, defer the earliest collision's losers on their owners, repeat.
    -> each rank's raw outputs of the final (collision-free) run."""
    global last_rounds
    for a in apps:
        a.shard_mode(query, 1)
    mode = 1
    for last_rounds in range(max_rounds):
        outs = [a.raw_outputs() for a in apps]
        fires = [a.sched_fires(query) for a in apps]
        if first_collision(np.concatenate(fires)) is None:
            return outs
        if mode == 1:                          # the resolution needs the notifyAt logs: re-run with them
            mode = 2
            for a in apps:
                a.shard_mode(query, 2)
            continue
        ops = [a.sched_ops(query) for a in apps]
        now, wait = _clock(apps[0], query)
        for r, key, tick, sched in resolve_collision(fires, ops, key_hash, now, wait):
            apps[r].sched_defer(query, key, tick, sched)
    raise RuntimeError("scheduler collision protocol did not converge")


def any_collision_dist(dist, fires: np.ndarray, device=None) -> bool:
    """True on every rank when two firings of any ranks (or of one rank) share (tick, scheduler, head): the
    collision test of the protocol's first round as a tensor exchange (all-gather of the (tick, sched, head)
    triples over the process group -- RCCL on the GPU ranks, gloo on CPU) and a sort on the rank's device,
    instead of pickled logs.  Every rank computes the same answer from the same gathered triples."""
    import torch
    world = dist.get_world_size()
    dev = torch.device("cpu") if device is None else device
    f = np.asarray(fires)
    trip = np.stack([f["tick"], f["sched"], f["head"]], 1).astype(np.int64) if len(f) else np.zeros((0, 3), np.int64)
    k = torch.from_numpy(np.ascontiguousarray(trip)).to(dev)
    cnt = torch.tensor([k.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    cs = [int(c.item()) for c in cnts]
    m = max(cs)
    if sum(cs) < 2:
        return False
    pad = torch.full((m, 3), -1, dtype=torch.int64, device=dev)
    pad[:k.shape[0]] = k
    got = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(got, pad)
    allk = torch.cat([g[:c] for g, c in zip(got, cs)])
    for col in (2, 1, 0):                       # lexicographic (tick, sched, head) by stable sorts
        allk = allk[torch.argsort(allk[:, col], stable=True)]
    return bool((allk[1:] == allk[:-1]).all(1).any().item())


def check_dictionaries(dist, app, n: int):
    """The protocol keys its replay by each rank's string ids (sched_fire / sched_op carry dictionary ids):
    every rank must have interned the same first `n` strings in the same order.  Raises otherwise."""
    import hashlib
    h = hashlib.sha256("\x00".join(app.string(i) for i in range(n)).encode()).hexdigest()
    box = [None] * dist.get_world_size()
    dist.all_gather_object(box, h)
    if any(b != h for b in box):
        raise RuntimeError("rank string dictionaries differ: the collision protocol needs identical key ids")


def settle_collisions_dist(dist, app, query: str, key_hash, max_rounds: int = 100_000, device=None,
                           collect=None):
    """The protocol across torch.distributed ranks (one app per rank): every round all-gathers the firing
    logs (and, once a collision was seen, the notifyAt logs); every rank computes the same resolution and
    defers its own losers.  -> this rank's outputs of the final run: `collect()` (default app.raw_outputs;
    bench.py passes a device-resident flush).  With `device`, the first round's collision test is the tensor
    exchange of any_collision_dist; the logs travel as objects only once a collision was found.

    Shard mode runs the whole stream from its first event at every round (batch mode: one push of the whole
    stream, then this protocol; a streaming caller re-settles the whole run per flush)."""
    world, me = dist.get_world_size(), dist.get_rank()
    collect = collect or app.raw_outputs
    global last_rounds
    app.shard_mode(query, 1)
    mode = 1
    for last_rounds in range(max_rounds):
        out = collect()
        mine = app.sched_fires(query)
        if mode == 1 and device is not None:
            if not any_collision_dist(dist, mine, device):
                return out
            mode = 2
            app.shard_mode(query, 2)
            continue
        fires = [None] * world
        dist.all_gather_object(fires, mine)
        if first_collision(np.concatenate(fires)) is None:
            return out
        if mode == 1:
            mode = 2
            app.shard_mode(query, 2)
            continue
        ops = [None] * world
        dist.all_gather_object(ops, app.sched_ops(query))
        now, wait = _clock(app, query)       # (every rank holds every tick: the same clocks)
        for r, key, tick, sched in resolve_collision(fires, ops, key_hash, now, wait):
            if r == me:
                app.sched_defer(query, key, tick, sched)
    raise RuntimeError("scheduler collision protocol did not converge")


# --------------------------------------------------------------------------------------------------------
# Streaming protocol (include/siddhi_gfx.h sg_query_shard_resolver, shard mode 3).
#
# The batch protocol above re-runs every rank from its first event per round, which is O(rounds x stream) and
# does not settle on natural streams.  In the streaming protocol each rank runs exactly as a single
# runtime does -- every flush from its settled base; after a collision the exact windowed sweep (nfa.hip
# NfaExec::sweep: each window from a checkpoint of the lane pools, only deferred instances re-run, the base moved
# to the sweep's end) -- and the two questions that runtime answers from its own Scheduler maps are asked of the
# driver instead, which answers from every rank's logs: is there a collision in this flush's run (kind 0), and
# which instances lose in this window (kind 1).  The maps live here, one replica per rank, at the ranks' common
# base, and advance over each window that settles.  Every rank asks the same questions in the same order (the
# windows are global tick ranges), so one all-gather per question keeps the ranks in step; a settled window is
# never run again, and a round re-runs only the deferred instances of one window.

def resolve_window(fires: Sequence[np.ndarray], ops: Sequence[np.ndarray], key_hash, tick_now, min_wait: int,
                   maps: dict):
    """One window of the streaming protocol over every rank's window logs (fires[r] / ops[r]), from `maps` (the
    Scheduler maps at the window's start, JdkHashMap per scheduler).  -> (losers, None) when the window holds a
    collision: [(rank, key, tick, sched)] to defer, as resolve_collision decides them (the same batching rule),
    `maps` untouched; ([], advanced maps) when it holds none: every notifyAt and every drained state's removal of
    the window applied in single-runtime order (nfa.hip NfaExec::replay_maps with resolve = false)."""
    import copy
    allf = np.concatenate([np.asarray(f) for f in fires]) if len(fires) else np.zeros(0)
    col = first_collision(allf) if len(allf) else None
    if col is None:
        work = maps
        cseq = None
    else:
        work = copy.deepcopy(maps)
        ctick, csched = col
        batch = tick_now is not None and min_wait > 0
        if batch:
            clock_end = int(tick_now[ctick]) + int(min_wait)
            last = int(np.searchsorted(np.asarray(tick_now), clock_end, side="left"))
            sel = allf["tick"] < last
            cseq = int(allf["seq"][sel].max()) if sel.any() else int(allf["seq"][(allf["tick"] == ctick)][0])
        else:
            cseq = int(allf["seq"][(allf["tick"] == ctick)][0])
    items = []
    for op in ops:
        op = np.asarray(op)
        if cseq is not None:
            op = op[op["seq"] <= cseq]
        for o in op.tolist():
            seq, head, key, tick, sub, pos, phase, kfire, ktarget = o[:9]
            if phase == 0:
                items.append((seq, 0, tick, kfire, 1, head, 0, sub, 1, ktarget, key))
            else:
                items.append((seq, 1, -1, -1, 1, 0, pos, sub, 1, ktarget, key))
    fired: dict = {}
    for r, f in enumerate(fires):
        for key, head, seq, tick, sched, empty_after, _p in np.asarray(f).tolist():
            fired.setdefault((tick, sched), []).append((r, key, head, empty_after, seq))
    for (tick, sched), fl in fired.items():
        seq = fl[0][4]
        if cseq is not None and seq > cseq:
            continue
        items.append((seq, 0, tick, sched, 0, -(1 << 63), 0, 0, 0, 0, 0))
        items.append((seq, 0, tick, sched, 2, (1 << 63) - 1, 0, 0, 2, 0, 0))
    items.sort(key=lambda t: t[:8])
    hcache: dict = {}

    def hk(key):
        h = hcache.get(key)
        if h is None:
            h = hcache[key] = key_hash(key)
        return h
    losers: list = []
    first = False
    dkeys: set = set()
    dheads: set = set()
    cap0: dict = {}
    smax: dict = {}
    for it in items:
        kind = it[8]
        if kind == 1:
            m = work.setdefault(it[9], JdkHashMap())
            m.touch(hk(it[10]), it[10])
            smax[it[9]] = max(smax.get(it[9], 0), m.size)
            continue
        tick, sched = it[2], it[3]
        fl = fired[(tick, sched)]
        m = work.setdefault(sched, JdkHashMap())
        if kind == 0:
            if cseq is None:
                continue
            if first:
                if int(tick_now[tick]) >= clock_end or any((r, key) in dkeys for r, key, _h, _e, _s in fl):
                    return losers, None
            elif (tick, sched) != (ctick, csched):
                continue
            byhead: dict = {}
            for r, key, head, _e, _s in fl:
                byhead.setdefault(head, []).append((r, key))
            shared = [h for h in sorted(byhead) if len(byhead[h]) >= 2]
            if first and shared:
                if len(m.tab) != cap0.get(sched, 0) or smax.get(sched, 0) + len(dkeys) + 1 > m.thr:
                    return losers, None
                if any((sched, h) in dheads for h in shared):
                    return losers, None
            for head in shared:
                grp = byhead[head]
                win = min(grp, key=lambda rk: m.rank(hk(rk[1]), rk[1]))
                for r, key in grp:
                    if (r, key) != win:
                        losers.append((r, key, tick, sched))
                        dkeys.add((r, key))
                        dheads.add((sched, head))
            if not first:
                first = True
                if not batch:
                    return losers, None
                cap0 = {k: len(v.tab) for k, v in work.items()}
                smax = {k: v.size for k, v in work.items()}
            continue
        for r, key, _head, empty_after, _s in fl:   # returnAllStates drops states with empty queues
            if empty_after and (r, key) not in dkeys:
                m.remove(hk(key), key)
    if cseq is None:
        return [], work
    if first:
        return losers, None
    raise RuntimeError("scheduler replay did not reach the collision")


class LocalGroup:
    """torch.distributed's get_rank / get_world_size / all_gather_object for rank threads of one process: the
    one-GPU rehearsal of the streaming protocol, whose ranks must flush concurrently (each flush waits inside the
    library for the others' logs).  bind(rank) in each rank's thread first."""

    def __init__(self, world: int, timeout: float = 300.0):
        import threading
        self.world = world
        self.box = [None] * world
        self.bar = threading.Barrier(world, timeout=timeout)
        self.local = threading.local()

    def bind(self, rank: int):
        self.local.rank = rank

    def get_rank(self) -> int:
        return self.local.rank

    def get_world_size(self) -> int:
        return self.world

    def all_gather_object(self, out: list, obj):
        self.bar.wait()
        self.box[self.local.rank] = obj
        self.bar.wait()
        out[:] = list(self.box)
        self.bar.wait()


class StreamingResolver:
    """The driver side of the streaming protocol for one rank's app (app.shard_resolver): answers the questions of
    the rank's flushes from every rank's logs (one all_gather_object per question over `dist`: a torch.distributed
    process group, RCCL on GPU ranks or gloo, or a LocalGroup) and keeps the Scheduler maps at the ranks' settled
    base.  rounds / windows / flushes count the collided rounds, settled windows and run checks."""

    def __init__(self, dist, app, query: str, key_hash):
        self.dist, self.app, self.query, self.key_hash = dist, app, query, key_hash
        self.maps: dict = {}
        self.rounds = self.windows = self.flushes = 0
        self.now, self.wait = None, 0
        app.shard_resolver(query, self)

    def reset(self):
        """After sg_reset: the ranks' base is the app's start again."""
        self.maps = {}
        self.rounds = self.windows = self.flushes = 0

    def _gather(self, obj) -> list:
        box = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(box, obj)
        return box

    def __call__(self, kind: int, fires: np.ndarray, ops: np.ndarray):
        if kind == 0:                      # a flush's run: the first collision across the ranks, if any
            self.flushes += 1
            if os.environ.get("SG_SHARD_ONE_PER_ROUND"):
                self.now, self.wait = None, 0
            else:
                self.now, self.wait = self.app.sched_clock(self.query)   # (the ticks do not change inside a flush)
            allf = np.concatenate(self._gather(fires))
            col = first_collision(allf) if len(allf) else None
            return (-1 if col is None else (col[0] << 8) | col[1]), []
        box_f, box_o = self._gather(fires), self._gather(ops)
        losers, adv = resolve_window(box_f, box_o, self.key_hash, self.now, self.wait, self.maps)
        if adv is not None:
            self.maps = adv
            self.windows += 1
            return 0, []
        self.rounds += 1
        me = self.dist.get_rank()
        return 1, [(key, tick, sched) for r, key, tick, sched in losers if r == me]
