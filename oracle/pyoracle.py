"""ctypes wrapper for the CPU restatement (oracle/_build/liboracle.so).

*** TEST INFRASTRUCTURE ONLY *** — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package `siddhi_amd`.

The API mirrors the reference's test idiom (TEST/query/pattern/EveryPatternTestCase.java etc.):
create an app from QL, register query / stream callbacks, send events through input handlers
(optionally sleeping — wall-clock tests are replayed with explicit virtual time), then read the
callbacks in the order the engine fired them.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the restatement with g++ (seconds)."""
    src = [os.path.join(_HERE, "siddhi_oracle.cpp")]
    os.makedirs(os.path.dirname(_LIB_PATH), exist_ok=True)
    newest = max(os.path.getmtime(p) for p in src + [os.path.join(_HERE, "..", "siddhi_amd", "csrc", "json.hpp")])
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < newest:
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", _LIB_PATH] + src
        subprocess.check_call(cmd)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.or_create.restype = C.c_void_p
        L.or_create.argtypes = [C.c_char_p]
        L.or_last_error.restype = C.c_char_p
        L.or_destroy.argtypes = [C.c_void_p]
        for f in ("or_stream_index", "or_query_index", "or_intern"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_char_p]
            getattr(L, f).restype = C.c_int
        L.or_string.argtypes = [C.c_void_p, C.c_int]
        L.or_string.restype = C.c_char_p
        L.or_add_query_callback.argtypes = [C.c_void_p, C.c_int]
        L.or_add_stream_callback.argtypes = [C.c_void_p, C.c_int]
        L.or_start.argtypes = [C.c_void_p]
        L.or_set_time.argtypes = [C.c_void_p, C.c_int64]
        L.or_send.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_send.restype = C.c_int
        L.or_out_ncb.argtypes = [C.c_void_p]
        L.or_out_ncb.restype = C.c_int64
        L.or_out_cbs.argtypes = [C.c_void_p] + [C.c_void_p] * 5
        L.or_out_nrows.argtypes = [C.c_void_p]
        L.or_out_nrows.restype = C.c_int64
        L.or_out_rows.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_out_clear.argtypes = [C.c_void_p]
        L.or_out_cb_seq.argtypes = [C.c_void_p, C.c_void_p]
        L.or_intern_range.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.or_send_chunks.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_int64, C.c_void_p, C.c_void_p]
        L.or_send_chunks.restype = C.c_int
        L.or_query_state_json.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int64]
        L.or_query_state_json.restype = C.c_int64
        _lib = L
    return _lib


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def encode_value(t: str, v: Any, intern) -> (int, int):
    """-> (raw int64 slot, isnull)"""
    if v is None:
        return 0, 1
    if t == "STRING":
        return intern(str(v)), 0
    if t in ("INT", "LONG"):
        return int(v), 0
    if t == "FLOAT":
        return struct.unpack("<I", struct.pack("<f", float(v)))[0], 0
    if t == "DOUBLE":
        return struct.unpack("<q", struct.pack("<d", float(v)))[0], 0
    if t == "BOOL":
        return int(bool(v)), 0
    raise ValueError(t)


def decode_value(t: str, raw: int, isnull: int, string_of):
    if isnull:
        return None
    raw = int(raw)
    if t == "STRING":
        return string_of(raw)
    if t == "INT":
        return int(np.int32(np.int64(raw)))
    if t == "LONG":
        return raw
    if t == "FLOAT":
        return struct.unpack("<f", struct.pack("<I", raw & 0xFFFFFFFF))[0]
    if t == "DOUBLE":
        return struct.unpack("<d", struct.pack("<q", raw))[0]
    if t == "BOOL":
        return bool(raw)
    return None


class OracleApp:
    """One SiddhiAppRuntime restated on the CPU."""

    def __init__(self, ql_or_desc):
        from siddhi_amd.ql import compile_app
        import json
        self.desc = compile_app(ql_or_desc) if isinstance(ql_or_desc, str) and not ql_or_desc.lstrip().startswith("{") \
            else (json.loads(ql_or_desc) if isinstance(ql_or_desc, str) else ql_or_desc)
        L = lib()
        self.L = L
        self.h = L.or_create(json.dumps(self.desc).encode())
        if not self.h:
            raise RuntimeError(L.or_last_error().decode())
        self.streams = {k: v for k, v in self.desc["streams"].items()}
        self.stream_names = list(self.desc["streams"].keys())
        self.queries = [q["name"] for q in self.desc["queries"]]
        self.now = 0
        self.playback = bool(self.desc.get("playback"))

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.L.or_destroy(self.h)
        except Exception:
            pass

    def intern(self, s: str) -> int:
        return self.L.or_intern(self.h, s.encode())

    def string(self, i: int) -> str:
        return self.L.or_string(self.h, int(i)).decode()

    def add_query_callback(self, name: str):
        qi = self.L.or_query_index(self.h, name.encode())
        if qi < 0:
            raise KeyError(name)
        self.L.or_add_query_callback(self.h, qi)

    def add_stream_callback(self, name: str):
        si = self.L.or_stream_index(self.h, name.encode())
        if si < 0:
            raise KeyError(name)
        self.L.or_add_stream_callback(self.h, si)

    def start(self):
        self.L.or_start(self.h)

    def sleep(self, ms: int):
        self.now += int(ms)
        if not self.playback:
            self.L.or_set_time(self.h, self.now)

    def set_time(self, t: int):
        self.now = int(t)
        self.L.or_set_time(self.h, self.now)

    def send(self, stream: str, data: Sequence[Any], ts: Optional[int] = None):
        self.send_many(stream, [(self.now if ts is None else ts, data)], batch=False)

    def send_many(self, stream: str, events: List, batch: bool):
        si = self.L.or_stream_index(self.h, stream.encode())
        types = [t for _n, t in self.streams[stream]]
        n = len(events)
        ts = np.empty(n, np.int64)
        raw = np.empty((n, len(types)), np.int64)
        nulls = np.zeros((n, len(types)), np.uint8)
        for i, (t, data) in enumerate(events):
            ts[i] = t
            for k, ty in enumerate(types):
                raw[i, k], nulls[i, k] = encode_value(ty, data[k], self.intern)
        self.send_columns(si, ts, raw, nulls, batch)

    def send_columns(self, si: int, ts: np.ndarray, raw: np.ndarray, nulls: Optional[np.ndarray], batch: bool):
        ts = np.ascontiguousarray(ts, np.int64)
        raw = np.ascontiguousarray(raw, np.int64)
        np_ = None if nulls is None else np.ascontiguousarray(nulls, np.uint8)
        rc = self.L.or_send(self.h, si, len(ts), ts.ctypes.data, raw.ctypes.data,
                            None if np_ is None else np_.ctypes.data, 1 if batch else 0)
        if rc != 0:
            raise RuntimeError(self.L.or_last_error().decode())

    def raw_outputs(self):
        """-> (cbs dict of arrays, ts[nrows], raw[nrows,width], nulls[nrows,width])"""
        L = self.L
        ncb = L.or_out_ncb(self.h)
        kind = np.empty(ncb, np.int32); target = np.empty(ncb, np.int32); cts = np.empty(ncb, np.int64)
        nin = np.empty(ncb, np.int32); nrm = np.empty(ncb, np.int32)
        if ncb:
            L.or_out_cbs(self.h, kind.ctypes.data, target.ctypes.data, cts.ctypes.data, nin.ctypes.data, nrm.ctypes.data)
        width = max([len(q["out_attrs"]) for q in self.desc["queries"]] +
                    [len(v) for v in self.streams.values()] + [1])
        nrows = L.or_out_nrows(self.h)
        ts = np.empty(nrows, np.int64); raw = np.empty((nrows, width), np.int64); nulls = np.empty((nrows, width), np.uint8)
        if nrows:
            L.or_out_rows(self.h, width, ts.ctypes.data, raw.ctypes.data, nulls.ctypes.data)
        return dict(kind=kind, target=target, ts=cts, n_in=nin, n_rm=nrm), ts, raw, nulls

    def outputs(self) -> List[Dict[str, Any]]:
        cbs, ts, raw, nulls = self.raw_outputs()
        out = []
        r = 0
        for i in range(len(cbs["kind"])):
            if cbs["kind"][i] == 0:
                q = self.desc["queries"][cbs["target"][i]]
                types = [t for _n, t in q["out_attrs"]]
                name = q["name"]
            else:
                name = self.stream_names[cbs["target"][i]]
                types = [t for _n, t in self.streams[name]]
            rows = []
            for part in ("in", "rm"):
                n = int(cbs["n_in"][i] if part == "in" else cbs["n_rm"][i])
                lst = []
                for _ in range(n):
                    lst.append([decode_value(t, raw[r, k], nulls[r, k], self.string) for k, t in enumerate(types)])
                    r += 1
                rows.append(lst)
            out.append({"kind": "query" if cbs["kind"][i] == 0 else "stream", "name": name,
                        "ts": int(cbs["ts"][i]), "in": rows[0], "rm": rows[1]})
        return out

    def clear_outputs(self):
        self.L.or_out_clear(self.h)

    def state_map(self, query: str):
        """StreamPreState.snapshot of every instance and pre-state processor (or_query_state_json)."""
        import json
        qi = self.L.or_query_index(self.h, query.encode())
        n = self.L.or_query_state_json(self.h, qi, None, 0)
        if n < 0:
            raise RuntimeError(self.L.or_last_error().decode())
        buf = C.create_string_buffer(n)
        self.L.or_query_state_json(self.h, qi, buf, n)
        return json.loads(buf.raw[:n])

    def callback_seq(self) -> np.ndarray:
        """Arrival index of the send whose processing fired each callback."""
        ncb = self.L.or_out_ncb(self.h)
        seq = np.empty(ncb, np.int64)
        if ncb:
            self.L.or_out_cb_seq(self.h, seq.ctypes.data)
        return seq


def sharded_run(ql, stream: str, ts: np.ndarray, raw: np.ndarray, shard_of: np.ndarray, nthreads: int,
                query: str = "query1", batch: bool = False, symbols: int = 0, shard_key=None):
    """Run a `partition with` app as `nthreads` key-disjoint oracle apps in parallel threads and merge
    their callbacks back into single-app order.

    Valid because partition instances never interact (PartitionStateHolder keys) for
    patterns without absent states: each shard gets the events of its keys in arrival order, and the
    callbacks are merged by the global arrival index of the send that fired them (a send belongs to
    one key, so one shard).  With batch=True the stream is one send(Event[]); `shard_key` (the
    partition key column, default shard_of) delimits its per-key runs.  Not valid for absent states or
    time windows (Scheduler state and clock advance are app-wide).  `raw` is the oracle row encoding (string ids from `symbols` interned
    "S0".."S{symbols-1}" first, identically in every shard).  Returns (raw outputs as
    OracleApp.raw_outputs, seconds spent in the shards).
    """
    import threading
    import time
    shards = [np.nonzero(shard_of == s)[0] for s in range(nthreads)]
    apps, outs = [], [None] * nthreads
    if batch:
        # one send(Event[]) of the whole stream is split by PartitionStreamReceiver into runs of
        # consecutive same-key events (PartitionStreamReceiver.java:176-217): each shard sends exactly
        # those runs, each tagged with the arrival index of its first event
        key = np.asarray(shard_key if shard_key is not None else shard_of)
        run0 = np.concatenate([[0], np.nonzero(key[1:] != key[:-1])[0] + 1]) if len(key) else np.zeros(0, np.int64)

    def work(s):
        a = apps[s]
        idx = shards[s]
        si = a.L.or_stream_index(a.h, stream.encode())
        if batch:
            mine = run0[shard_of[run0] == s]
            starts = np.searchsorted(idx, mine).astype(np.int64)
            starts = np.ascontiguousarray(np.concatenate([starts, [len(idx)]]), np.int64)
            seqs = np.ascontiguousarray(mine, np.int64)
            t_ = np.ascontiguousarray(ts[idx], np.int64)
            r_ = np.ascontiguousarray(raw[idx], np.int64)
            rc = a.L.or_send_chunks(a.h, si, len(idx), t_.ctypes.data, r_.ctypes.data, None, len(mine),
                                    starts.ctypes.data, seqs.ctypes.data)
            if rc != 0:
                raise RuntimeError(a.L.or_last_error().decode())
            outs[s] = (a.raw_outputs(), a.callback_seq())
        else:
            a.send_columns(si, ts[idx], raw[idx], None, False)
            cbs = a.raw_outputs()
            outs[s] = (cbs, idx[a.callback_seq()] if len(cbs[0]["kind"]) else np.zeros(0, np.int64))

    for s in range(nthreads):
        a = OracleApp(ql)
        a.add_query_callback(query)
        a.start()
        if symbols:
            a.L.or_intern_range(a.h, b"S", int(symbols))
        apps.append(a)
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(s,)) for s in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    secs = time.perf_counter() - t0
    # merge: callback c of shard s was fired by global event shards[s][seq]
    keys, parts = [], []
    for s in range(nthreads):
        (cbs, rts, rraw, rnul), g = outs[s]
        keys.append(g)
        nrow = (cbs["n_in"] + cbs["n_rm"]).astype(np.int64)
        parts.append((cbs, rts, rraw, rnul, nrow, np.concatenate([[0], np.cumsum(nrow)])))
    allk = np.concatenate(keys)
    order = np.argsort(allk, kind="stable")
    fields = ("kind", "target", "ts", "n_in", "n_rm")
    cbs = {f: np.concatenate([parts[s][0][f] for s in range(nthreads)])[order] for f in fields}
    # rows: concatenate every shard's rows, then gather the merged callbacks' row ranges
    base = np.concatenate([[0], np.cumsum([len(parts[s][1]) for s in range(nthreads)])])
    starts = np.concatenate([base[s] + parts[s][5][:-1] for s in range(nthreads)])[order]
    lens = np.concatenate([parts[s][4] for s in range(nthreads)])[order]
    tot = int(lens.sum())
    idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(tot)
    rts = np.concatenate([parts[s][1] for s in range(nthreads)])[idx]
    rraw = np.concatenate([parts[s][2] for s in range(nthreads)])[idx]
    rnul = np.concatenate([parts[s][3] for s in range(nthreads)])[idx]
    return (cbs, rts, rraw, rnul), secs
