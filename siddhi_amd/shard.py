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
