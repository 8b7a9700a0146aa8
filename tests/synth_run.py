"""Drive the oracle and the GPU path with the same synthetic columnar stream."""
import numpy as np

from siddhi_amd import synth


def intern_symbols(engine, k):
    """Intern "S0".."S{k-1}"; returns the id of each symbol index in `engine`'s dictionary."""
    return np.array([engine.intern(f"S{i}") for i in range(k)], np.int32)


def oracle_feed(app, stream, d, ids, batch=True, chunk=None):
    from oracle.pyoracle import encode_value  # noqa: F401  (test infrastructure)
    si = app.L.or_stream_index(app.h, stream.encode())
    n = len(d["ts"])
    raw = np.empty((n, 3), np.int64)
    raw[:, 0] = ids[d["symbol"]]
    raw[:, 1] = d["price"].view(np.uint32).astype(np.int64)
    raw[:, 2] = d["volume"].astype(np.int64)
    step = chunk or n
    for s in range(0, n, step):
        app.send_columns(si, d["ts"][s:s + step], raw[s:s + step], None, batch)


def gpu_feed(app, stream, d, ids, batch=True, chunk=None):
    n = len(d["ts"])
    step = chunk or n
    sym = ids[d["symbol"]]
    for s in range(0, n, step):
        app.send_columns(stream, d["ts"][s:s + step], [sym[s:s + step], d["price"][s:s + step],
                                                      d["volume"][s:s + step]], batch)


def compare_raw(o, g, ncols):
    """Compare (cbs, ts, raw, nulls) tuples from the oracle and the GPU engine."""
    ocb, ots, oraw, onul = o
    gcb, gts, graw, gnul = g
    for k in ("kind", "target", "ts", "n_in", "n_rm"):
        assert np.array_equal(ocb[k], gcb[k]), f"callback field {k} differs " \
            f"(oracle {len(ocb[k])} callbacks, gpu {len(gcb[k])})"
    assert np.array_equal(ots, gts)
    assert np.array_equal(onul[:, :ncols], gnul[:, :ncols])
    m = onul[:, :ncols] == 0
    assert np.array_equal(np.where(m, oraw[:, :ncols], 0), np.where(m, graw[:, :ncols], 0))


def raw_matrix(types, cols):
    """Oracle row encoding of typed columns: int sign-extended, float32/float64 bits, long, string id."""
    n = len(cols[0]) if cols else 0
    raw = np.empty((n, len(cols)), np.int64)
    for k, (t, c) in enumerate(zip(types, cols)):
        if t == "FLOAT":
            raw[:, k] = np.asarray(c, np.float32).view(np.uint32).astype(np.int64)
        elif t == "DOUBLE":
            raw[:, k] = np.asarray(c, np.float64).view(np.int64)
        else:
            raw[:, k] = np.asarray(c).astype(np.int64)
    return raw


def feed_both(o, g, stream, types, ts, cols, batch=True, chunk=None, flush_each=False, after=None):
    """Send the same typed columns (strings already interned to the same ids) to both engines; `after()`
    runs after each chunk's flush."""
    si = o.L.or_stream_index(o.h, stream.encode())
    raw = raw_matrix(types, cols)
    n = len(ts)
    step = chunk or max(n, 1)
    for s in range(0, n, step):
        o.send_columns(si, ts[s:s + step], raw[s:s + step], None, batch)
        g.send_columns(stream, ts[s:s + step], [c[s:s + step] for c in cols], batch)
        if flush_each:
            g.flush()
            if after:
                after()
