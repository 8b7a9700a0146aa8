"""Host-side mirror of Siddhi's public API over the C ABI (include/siddhi_gfx.h).

    SiddhiManager().createSiddhiAppRuntime(ql)    CORE/SiddhiManager.java:94-97
    SiddhiAppRuntime.getInputHandler / addCallback / start / shutdown
                                                  CORE/SiddhiAppRuntime.java:116-167
    InputHandler.send(Object[]) / send(ts, Object[]) / send(Event[])
                                                  CORE/stream/input/InputHandler.java:50-94
    QueryCallback.receive(ts, inEvents, removeEvents)  CORE/query/output/callback/QueryCallback.java:61-91
    StreamCallback.receive(events)                CORE/stream/output/StreamCallback.java:93-104

Every query runs on the MI355X through libsiddhi_gfx.so; there is no CPU fallback in this
package.  If the library is missing or the GPU path rejects a query, construction raises.
Callbacks fire when the runtime is flushed (explicitly, on `flush()`/`shutdown()`, or after every
send when `auto_flush=True`), in the order the reference would fire them.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import struct
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .ql import compile_app

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SG_LIB") or os.path.join(_HERE, "_build", "libsiddhi_gfx.so")   # SG_LIB: tuning hook (an alternative build)
_lib = None

# include/siddhi_gfx.h sg_sched_fire / sg_sched_op
SCHED_FIRE = np.dtype([("key", "<i8"), ("head", "<i8"), ("seq", "<i8"), ("tick", "<i4"), ("sched", "i1"),
                       ("empty_after", "i1"), ("pad", "<i2")])
SCHED_OP = np.dtype([("seq", "<i8"), ("head", "<i8"), ("key", "<i8"), ("tick", "<i4"), ("sub", "<i4"),
                     ("pos", "<i4"), ("phase", "i1"), ("kfire", "i1"), ("ktarget", "i1"), ("pad", "i1")])

TYPE_CODES = {"STRING": 0, "INT": 1, "LONG": 2, "FLOAT": 3, "DOUBLE": 4, "BOOL": 5}
NP_TYPES = {"STRING": np.int32, "INT": np.int32, "LONG": np.int64, "FLOAT": np.float32,
            "DOUBLE": np.float64, "BOOL": np.uint8}
PATHS = {1: "followed_by", 2: "nfa", 3: "window_agg", 4: "keyed_followed_by", 5: "window", -2: "unsupported"}


class SiddhiGfxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class _Batch(C.Structure):
    _fields_ = [("n", C.c_int64), ("ts", C.c_void_p), ("cols", C.c_void_p), ("nulls", C.c_void_p),
                ("batch", C.c_int), ("seq", C.c_void_p)]


class _Options(C.Structure):
    _fields_ = [("device", C.c_int), ("capacity", C.c_int64)]


def lib():
    """Load the in-tree HIP library; fail loudly if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: run `python -m siddhi_amd.build` "
                              "(hipcc --offload-arch=gfx950) first; there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        L.sg_last_error.restype = C.c_char_p
        L.sg_app_create.argtypes = [C.c_char_p, C.c_void_p, C.POINTER(C.c_void_p)]
        L.sg_app_destroy.argtypes = [C.c_void_p]
        for f in ("sg_stream_index", "sg_query_index", "sg_intern"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_char_p]
        L.sg_string.argtypes = [C.c_void_p, C.c_int]
        L.sg_string.restype = C.c_char_p
        L.sg_query_path.argtypes = [C.c_void_p, C.c_int]
        L.sg_query_unsupported_reason.argtypes = [C.c_void_p, C.c_int]
        L.sg_query_unsupported_reason.restype = C.c_char_p
        L.sg_query_count.argtypes = [C.c_void_p]
        L.sg_stream_count.argtypes = [C.c_void_p]
        L.sg_add_query_callback.argtypes = [C.c_void_p, C.c_int]
        L.sg_add_stream_callback.argtypes = [C.c_void_p, C.c_int]
        L.sg_start.argtypes = [C.c_void_p]
        L.sg_reset.argtypes = [C.c_void_p]
        L.sg_snapshot.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_int64)]
        L.sg_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.sg_free_buffer.argtypes = [C.c_void_p]
        L.sg_push.argtypes = [C.c_void_p, C.c_int, C.POINTER(_Batch)]
        L.sg_push_device.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.sg_push_device_seq.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_int, C.c_void_p]
        L.sg_advance_time.argtypes = [C.c_void_p, C.c_int64]
        L.sg_set_halo.argtypes = [C.c_void_p, C.c_int, C.c_int64]
        L.sg_flush.argtypes = [C.c_void_p]
        L.sg_flush_device.argtypes = [C.c_void_p, C.c_void_p]
        L.sg_out_ncallbacks.argtypes = [C.c_void_p]
        L.sg_out_ncallbacks.restype = C.c_int64
        L.sg_out_callbacks.argtypes = [C.c_void_p] + [C.c_void_p] * 5
        L.sg_out_nrows.argtypes = [C.c_void_p]
        L.sg_out_nrows.restype = C.c_int64
        L.sg_out_rows.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sg_out_clear.argtypes = [C.c_void_p]
        L.sg_out_callback_seq.argtypes = [C.c_void_p, C.c_void_p]
        L.sg_out_callback_tick.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.sg_push_shard.argtypes = [C.c_void_p, C.c_int, C.POINTER(_Batch), C.c_int64, C.c_void_p, C.c_int64]
        L.sg_last_match_count.argtypes = [C.c_void_p, C.c_int]
        L.sg_last_match_count.restype = C.c_int64
        L.sg_last_kernel_ms.argtypes = [C.c_void_p, C.c_char_p]
        L.sg_last_kernel_ms.restype = C.c_double
        L.sg_query_buffered.argtypes = [C.c_void_p, C.c_int]
        L.sg_query_buffered.restype = C.c_int64
        L.sg_query_kernel_source.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int64]
        L.sg_query_kernel_source.restype = C.c_int64
        L.sg_query_compile.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]
        L.sg_query_shard_mode.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.sg_query_sched_fires.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        L.sg_query_sched_fires.restype = C.c_int64
        L.sg_query_sched_clock.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p]
        L.sg_query_sched_clock.restype = C.c_int64
        L.sg_query_sched_ops.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        L.sg_query_sched_ops.restype = C.c_int64
        L.sg_query_sched_defer.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int32, C.c_int32]
        L.sg_query_shard_resolver.argtypes = [C.c_void_p, C.c_int, SHARD_RESOLVER, C.c_void_p]
        L.sg_query_state_json.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int64]
        L.sg_query_state_json.restype = C.c_int64
        _lib = L
    return _lib


# include/siddhi_gfx.h sg_shard_resolver_fn
SHARD_RESOLVER = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                             C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64))


def _check(rc: int):
    if rc < 0:
        raise SiddhiGfxError(rc, lib().sg_last_error().decode())
    return rc


def _decode(t: str, raw: int, isnull: int, string_of):
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


class Event:
    """io.siddhi.core.event.Event"""

    def __init__(self, timestamp: int, data: List[Any], is_expired: bool = False):
        self.timestamp = timestamp
        self.data = data
        self.is_expired = is_expired

    def getData(self, i: Optional[int] = None):
        return self.data if i is None else self.data[i]

    def getTimestamp(self):
        return self.timestamp

    def __repr__(self):
        return f"Event{{timestamp={self.timestamp}, data={self.data}, isExpired={self.is_expired}}}"


class QueryCallback:
    def receive(self, timestamp: int, in_events: Optional[List[Event]], remove_events: Optional[List[Event]]):
        raise NotImplementedError


class StreamCallback:
    def receive(self, events: List[Event]):
        raise NotImplementedError


class GpuApp:
    """One SiddhiAppRuntime on the GPU path — low-level handle over the C ABI."""

    def __init__(self, ql_or_desc, device: int = 0, allow_partial: bool = False):
        """allow_partial=False (the tests' default) raises SiddhiGfxError(-2) when any query of the app is
        not lowered to the device; the library itself keeps such queries as SG_E_UNSUPPORTED for the shim."""
        self.desc = compile_app(ql_or_desc) if isinstance(ql_or_desc, str) else ql_or_desc
        L = lib()
        self.L = L
        h = C.c_void_p()
        opts = _Options(device, 0)
        _check(L.sg_app_create(json.dumps(self.desc).encode(), C.byref(opts), C.byref(h)))
        self.h = h
        self.unsupported = {}
        for qi, q in enumerate(self.desc["queries"]):
            r = L.sg_query_unsupported_reason(h, qi)
            if r is not None:
                self.unsupported[q["name"]] = r.decode()
        if self.unsupported and not allow_partial:
            msg = "; ".join(f"query '{k}': {v}" for k, v in self.unsupported.items())
            L.sg_app_destroy(h)
            self.h = None
            raise SiddhiGfxError(-2, msg)
        self.streams = dict(self.desc["streams"])
        self.stream_names = list(self.streams.keys())
        self.queries = [q["name"] for q in self.desc["queries"]]
        self.playback = bool(self.desc.get("playback"))
        self.now = 0
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            self.L.sg_app_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def path(self, query: str) -> str:
        return PATHS.get(self.L.sg_query_path(self.h, self.queries.index(query)), "?")

    def intern(self, s: str) -> int:
        return self.L.sg_intern(self.h, s.encode())

    def string(self, i: int) -> str:
        r = self.L.sg_string(self.h, int(i))
        return None if r is None else r.decode()

    def add_query_callback(self, name: str):
        _check(self.L.sg_add_query_callback(self.h, _check(self.L.sg_query_index(self.h, name.encode()))))

    def add_stream_callback(self, name: str):
        _check(self.L.sg_add_stream_callback(self.h, _check(self.L.sg_stream_index(self.h, name.encode()))))

    def start(self):
        _check(self.L.sg_start(self.h))

    def reset(self):
        _check(self.L.sg_reset(self.h))

    def snapshot(self) -> bytes:
        """SiddhiAppRuntime.snapshot(): flush, then the state of every query as bytes (sg_snapshot)."""
        p = C.POINTER(C.c_uint8)()
        n = C.c_int64(0)
        _check(self.L.sg_snapshot(self.h, C.byref(p), C.byref(n)))
        try:
            return C.string_at(p, n.value)
        finally:
            self.L.sg_free_buffer(p)

    def restore(self, state: bytes):
        """SiddhiAppRuntime.restore(byte[]) into an app created from the same descriptor (sg_restore)."""
        buf = C.create_string_buffer(state, len(state))
        _check(self.L.sg_restore(self.h, buf, len(state)))

    def set_halo(self, stream: str, n_halo: int):
        """The last n_halo events pushed to `stream` are the next rank's leading events (multi-GPU split
        of an unkeyed followed-by): they complete this range's partials but start none (sg_set_halo)."""
        si = _check(self.L.sg_stream_index(self.h, stream.encode()))
        _check(self.L.sg_set_halo(self.h, si, int(n_halo)))

    def sleep(self, ms: int):
        self.now += int(ms)
        _check(self.L.sg_advance_time(self.h, self.now))

    def set_time(self, t: int):
        self.now = int(t)
        _check(self.L.sg_advance_time(self.h, self.now))

    def send(self, stream: str, data: Sequence[Any], ts: Optional[int] = None):
        self.send_many(stream, [(self.now if ts is None else ts, data)], batch=False)

    def send_many(self, stream: str, events: List, batch: bool):
        """`events`: [(ts, [values])]; a None value is a null attribute (sent as a null flag)."""
        types = [t for _n, t in self.streams[stream]]
        cols = []
        nulls = np.array([[v is None for v in d] for _t, d in events], np.uint8).reshape(len(events), len(types))
        for k, t in enumerate(types):
            if t == "STRING":
                cols.append(np.array([0 if d[k] is None else self.intern(str(d[k])) for _t, d in events], np.int32))
            else:
                cols.append(np.array([0 if d[k] is None else d[k] for _t, d in events], NP_TYPES[t]))
        ts = np.array([t for t, _d in events], np.int64)
        self.send_columns(stream, ts, cols, batch, nulls=nulls if nulls.any() else None)

    def send_columns(self, stream: str, ts: np.ndarray, cols: List[np.ndarray], batch: bool, seq=None,
                     nulls: Optional[np.ndarray] = None):
        """`seq`: optional global arrival index of each event (events routed to this rank's keys);
        `nulls`: optional [n, arity] null flags."""
        si = _check(self.L.sg_stream_index(self.h, stream.encode()))
        ts = np.ascontiguousarray(ts, np.int64)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        sq = None if seq is None else np.ascontiguousarray(seq, np.int64)
        nl = None if nulls is None else np.ascontiguousarray(nulls, np.uint8)
        b = _Batch(len(ts), ts.ctypes.data, C.cast(ptrs, C.c_void_p), None if nl is None else nl.ctypes.data,
                   1 if batch else 0, None if sq is None else sq.ctypes.data)
        _check(self.L.sg_push(self.h, si, C.byref(b)))

    def push_shard(self, stream: str, ts: np.ndarray, cols: List[np.ndarray], seq: np.ndarray,
                   global_ts: np.ndarray, seq0: int = 0, batch: bool = False):
        """This rank's share of one global send (sg_push_shard): the events it owns (`seq`: their global
        arrival indices) and the global send's timestamps, which advance the playback clock on every rank."""
        si = _check(self.L.sg_stream_index(self.h, stream.encode()))
        ts = np.ascontiguousarray(ts, np.int64)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        sq = np.ascontiguousarray(seq, np.int64)
        gt = np.ascontiguousarray(global_ts, np.int64)
        b = _Batch(len(ts), ts.ctypes.data, C.cast(ptrs, C.c_void_p), None, 1 if batch else 0, sq.ctypes.data)
        _check(self.L.sg_push_shard(self.h, si, C.byref(b), len(gt), gt.ctypes.data, seq0))

    def push_device(self, stream: str, n: int, ts_ptr: int, col_ptrs: List[int], hip_stream: int = 0,
                    batch: bool = True, seq_ptr: int = 0):
        """Adopt device-resident columns; `seq_ptr`: optional device int64 global arrival indices."""
        si = _check(self.L.sg_stream_index(self.h, stream.encode()))
        arr = (C.c_void_p * len(col_ptrs))(*col_ptrs)
        self._keep.append(arr)
        hs = C.c_void_p(hip_stream) if hip_stream else None
        if seq_ptr:
            _check(self.L.sg_push_device_seq(self.h, si, n, C.c_void_p(ts_ptr), C.cast(arr, C.c_void_p),
                                             C.c_void_p(seq_ptr), 1 if batch else 0, hs))
        else:
            _check(self.L.sg_push_device(self.h, si, n, C.c_void_p(ts_ptr), C.cast(arr, C.c_void_p),
                                         1 if batch else 0, hs))

    def flush(self):
        _check(self.L.sg_flush(self.h))

    def flush_device(self, hip_stream: int = 0):
        _check(self.L.sg_flush_device(self.h, C.c_void_p(hip_stream) if hip_stream else None))

    def match_count(self, query: str) -> int:
        return int(self.L.sg_last_match_count(self.h, self.queries.index(query)))

    def buffered(self, query: str) -> int:
        """Events the query still holds after its last flush (-1: not tracked on its path)."""
        return int(self.L.sg_query_buffered(self.h, self.queries.index(query)))

    # cross-rank Scheduler collisions (include/siddhi_gfx.h sg_query_shard_mode; driver: shard.py)
    def shard_mode(self, query: str, mode: int):
        _check(self.L.sg_query_shard_mode(self.h, self.queries.index(query), mode))

    def sched_fires(self, query: str) -> np.ndarray:
        """The last flush's Scheduler firings (shard mode) as a SCHED_FIRE record array."""
        q = self.queries.index(query)
        c = _check(self.L.sg_query_sched_fires(self.h, q, None, 0))
        out = np.zeros(c, SCHED_FIRE)
        if c:
            _check(self.L.sg_query_sched_fires(self.h, q, out.ctypes.data, c))
        return out

    def sched_ops(self, query: str) -> np.ndarray:
        """The last flush's Scheduler.notifyAt log (shard mode 2) as a SCHED_OP record array."""
        q = self.queries.index(query)
        c = _check(self.L.sg_query_sched_ops(self.h, q, None, 0))
        out = np.zeros(c, SCHED_OP)
        if c:
            _check(self.L.sg_query_sched_ops(self.h, q, out.ctypes.data, c))
        return out

    def sched_clock(self, query: str):
        """(clock of every Scheduler tick so far, shortest absent wait): the driver's batching bound."""
        q = self.queries.index(query)
        w = C.c_int64(0)
        c = _check(self.L.sg_query_sched_clock(self.h, q, None, 0, C.addressof(w)))
        now = np.zeros(c, np.int64)
        if c:
            _check(self.L.sg_query_sched_clock(self.h, q, now.ctypes.data, c, None))
        return now, int(w.value)

    def shard_resolver(self, query: str, resolve):
        """Streaming shard mode (sg_query_shard_resolver): `resolve(kind, fires, ops) -> (code, [(key, tick, sched)])`
        answers the rank's Scheduler-map questions during its flushes (siddhi_amd/shard.py StreamingResolver)."""
        import traceback

        def arr(p, n, dt):
            if not n:
                return np.zeros(0, dt)
            return np.frombuffer((C.c_char * (n * dt.itemsize)).from_address(p), dt).copy()

        def cb(_user, kind, fp, nf, op, no, dout, cap, nd):
            try:
                code, losers = resolve(int(kind), arr(fp, nf, SCHED_FIRE), arr(op, no, SCHED_OP))
                if len(losers) > cap:
                    return -2
                for i, (key, tick, sched) in enumerate(losers):
                    dout[3 * i], dout[3 * i + 1], dout[3 * i + 2] = int(key), int(tick), int(sched)
                nd[0] = len(losers)
                return int(code)
            except Exception:
                traceback.print_exc()
                return -2
        f = SHARD_RESOLVER(cb)
        self._keep.append(f)            # (the library holds the pointer for the app's life)
        _check(self.L.sg_query_shard_resolver(self.h, self.queries.index(query), f, None))

    def sched_defer(self, query: str, key: int, tick: int, sched: int):
        _check(self.L.sg_query_sched_defer(self.h, self.queries.index(query), int(key), int(tick), int(sched)))

    def state_map(self, query: str):
        """The pattern state after the last flush in StreamPreState.snapshot's shape (sg_query_state_json)."""
        import json
        q = self.queries.index(query)
        n = _check(self.L.sg_query_state_json(self.h, q, None, 0))
        buf = C.create_string_buffer(max(n, 1))
        _check(self.L.sg_query_state_json(self.h, q, buf, n))
        return json.loads(buf.raw[:n])

    def kernel_source(self, query: str) -> str:
        """The generated source of the query's run-time compiled kernel (NFA path; nfa_rtc.hpp)."""
        q = self.queries.index(query)
        n = int(self.L.sg_query_kernel_source(self.h, q, None, 0))
        if n < 0:
            _check(n)
        buf = C.create_string_buffer(n + 1)
        self.L.sg_query_kernel_source(self.h, q, buf, n + 1)
        return buf.value.decode()

    def compile_kernel(self, query: str):
        """Compile the query's kernel into the code-object cache now (no GPU needed; releases the GIL, so apps can
        compile in parallel threads) -> (hipRTC ms, found in the disk cache)."""
        ms, disk = C.c_double(0), C.c_int(0)
        _check(self.L.sg_query_compile(self.h, self.queries.index(query), C.byref(ms), C.byref(disk)))
        return ms.value, bool(disk.value)

    def kernel_ms(self, name: str) -> float:
        return float(self.L.sg_last_kernel_ms(self.h, name.encode()))

    def _out_arrays(self, reuse, name, n, dtype, width=None):
        """A fresh array, or (reuse) a view of one kept on the app and grown by doubling: the JNI drain's
        direct buffers are reused the same way, so a drain does not page in new memory every time."""
        shape = (n,) if width is None else (n, width)
        if not reuse:
            return np.empty(shape, dtype)
        cache = self.__dict__.setdefault("_drain_cache", {})
        a = cache.get(name)
        if a is None or a.shape[0] < n or a.shape[1:] != shape[1:]:
            cap = max(n, 2 * a.shape[0] if a is not None and a.shape[1:] == shape[1:] else n)
            a = cache[name] = np.empty((cap,) + shape[1:], dtype)
        return a[:n]

    def raw_outputs(self, width: Optional[int] = None, reuse: bool = False):
        """Flush; -> (callback arrays, ts[nrows], raw[nrows,width], nulls[nrows,width]) and clear.
        reuse=True returns views of arrays the app keeps and overwrites at the next reuse call."""
        self.flush()
        L = self.L
        ncb = L.sg_out_ncallbacks(self.h)
        ar = lambda name, n, dt, w=None: self._out_arrays(reuse, name, n, dt, w)
        kind = ar("kind", ncb, np.int32); target = ar("target", ncb, np.int32); cts = ar("cts", ncb, np.int64)
        nin = ar("nin", ncb, np.int32); nrm = ar("nrm", ncb, np.int32)
        if ncb:
            _check(L.sg_out_callbacks(self.h, kind.ctypes.data, target.ctypes.data, cts.ctypes.data,
                                      nin.ctypes.data, nrm.ctypes.data))
        if width is None:
            width = max([len(q["out_attrs"]) for q in self.desc["queries"]] +
                        [len(v) for v in self.streams.values()] + [1])
        nrows = L.sg_out_nrows(self.h)
        ts = ar("ts", nrows, np.int64); raw = ar("raw", nrows, np.int64, width)
        nulls = ar("nulls", nrows, np.uint8, width)
        if nrows:
            _check(L.sg_out_rows(self.h, width, ts.ctypes.data, raw.ctypes.data, nulls.ctypes.data))
        seq = ar("seq", ncb, np.int64)
        tsched = ar("tsched", ncb, np.int32)
        tdl = ar("tdl", ncb, np.int64)
        if ncb:
            _check(L.sg_out_callback_seq(self.h, seq.ctypes.data))
            _check(L.sg_out_callback_tick(self.h, tsched.ctypes.data, tdl.ctypes.data))
        _check(L.sg_out_clear(self.h))
        return (dict(kind=kind, target=target, ts=cts, n_in=nin, n_rm=nrm, seq=seq, tsched=tsched, tdl=tdl),
                ts, raw, nulls)

    def outputs(self) -> List[Dict[str, Any]]:
        """Flush, then return the callbacks fired since the previous outputs() / raw_outputs() call (same
        shape as oracle.pyoracle); the native buffer is cleared, nothing is retained here."""
        self.flush()
        L = self.L
        ncb = L.sg_out_ncallbacks(self.h)
        kind = np.empty(ncb, np.int32); target = np.empty(ncb, np.int32); cts = np.empty(ncb, np.int64)
        nin = np.empty(ncb, np.int32); nrm = np.empty(ncb, np.int32)
        if ncb:
            _check(L.sg_out_callbacks(self.h, kind.ctypes.data, target.ctypes.data, cts.ctypes.data,
                                      nin.ctypes.data, nrm.ctypes.data))
        width = max([len(q["out_attrs"]) for q in self.desc["queries"]] +
                    [len(v) for v in self.streams.values()] + [1])
        nrows = L.sg_out_nrows(self.h)
        ts = np.empty(nrows, np.int64); raw = np.empty((nrows, width), np.int64)
        nulls = np.empty((nrows, width), np.uint8)
        if nrows:
            _check(L.sg_out_rows(self.h, width, ts.ctypes.data, raw.ctypes.data, nulls.ctypes.data))
        out, r = [], 0
        for i in range(ncb):
            if kind[i] == 0:
                q = self.desc["queries"][target[i]]
                types = [t for _n, t in q["out_attrs"]]
                name = q["name"]
            else:
                name = self.stream_names[target[i]]
                types = [t for _n, t in self.streams[name]]
            rows = []
            for n in (int(nin[i]), int(nrm[i])):
                lst = []
                for _ in range(n):
                    lst.append([_decode(t, raw[r, k], nulls[r, k], self.string) for k, t in enumerate(types)])
                    r += 1
                rows.append(lst)
            out.append({"kind": "query" if kind[i] == 0 else "stream", "name": name, "ts": int(cts[i]),
                        "in": rows[0], "rm": rows[1]})
        _check(L.sg_out_clear(self.h))
        return out


class InputHandler:
    def __init__(self, rt: "SiddhiAppRuntime", stream: str):
        self._rt = rt
        self.stream = stream

    def getStreamId(self):
        return self.stream

    def send(self, *args):
        """send(Object[]) | send(long ts, Object[]) | send(Event) | send(Event[])"""
        rt = self._rt
        if len(args) == 2:
            rt.app.send(self.stream, list(args[1]), int(args[0]))
        elif isinstance(args[0], Event):
            rt.app.send(self.stream, list(args[0].data), args[0].timestamp)
        elif args[0] and isinstance(args[0][0], Event):
            rt.app.send_many(self.stream, [(e.timestamp, list(e.data)) for e in args[0]], batch=True)
        else:
            rt.app.send(self.stream, list(args[0]), None)
        if rt.auto_flush:
            rt.flush()


class SiddhiAppRuntime:
    def __init__(self, ql: str, auto_flush: bool = False, device: int = 0):
        self.app = GpuApp(ql, device)
        self.auto_flush = auto_flush
        self._qcb: Dict[str, List[QueryCallback]] = {}
        self._scb: Dict[str, List[StreamCallback]] = {}

    def getInputHandler(self, stream: str) -> InputHandler:
        if stream not in self.app.streams:
            raise KeyError(stream)
        return InputHandler(self, stream)

    def addCallback(self, name: str, cb):
        if isinstance(cb, QueryCallback):
            self.app.add_query_callback(name)
            self._qcb.setdefault(name, []).append(cb)
        else:
            self.app.add_stream_callback(name)
            self._scb.setdefault(name, []).append(cb)

    def start(self):
        self.app.start()

    def flush(self):
        for o in self.app.outputs():
            if o["kind"] == "query":
                ins = [Event(o["ts"], r) for r in o["in"]] or None
                rms = [Event(o["ts"], r, True) for r in o["rm"]] or None
                for cb in self._qcb.get(o["name"], []):
                    cb.receive(o["ts"], ins, rms)
            else:
                evs = [Event(o["ts"], r) for r in o["in"]]
                for cb in self._scb.get(o["name"], []):
                    cb.receive(evs)

    def snapshot(self) -> bytes:
        self.flush()
        return self.app.snapshot()

    def restore(self, state: bytes):
        self.app.restore(state)

    def shutdown(self):
        self.flush()
        self.app.close()


class SiddhiManager:
    """io.siddhi.core.SiddhiManager restricted to the device path."""

    def createSiddhiAppRuntime(self, ql: str, auto_flush: bool = False) -> SiddhiAppRuntime:
        return SiddhiAppRuntime(ql, auto_flush=auto_flush)

    def shutdown(self):
        pass
