"""The device window path (window_dev.hpp, GenWindowExec::flush_device) against the oracle, flushing every few
dozen events so that every flush starts from the window state the previous one carried (held rows of the
length / lengthBatch / time queues, pending batches, the RESET copy, aggregator states).  Each flush that had
events must have run on the device (kernel_ms "gw_device" == 1).  Bar: bit-exact rows, timestamps and
callback grouping vs the oracle's QueryCallbacks (LengthWindowProcessor.java:106-141,
LengthBatchWindowProcessor.java:154-351, TimeWindowProcessor.java:133-169, QuerySelector.java:76-374)."""
import numpy as np
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import compare_raw, intern_symbols, raw_matrix

pytestmark = pytest.mark.gpu

S = synth.STOCK_STREAM
TYPES = ["STRING", "FLOAT", "INT"]

SINGLE = {
    "length_all_events": "from StockStream#window.length(5) select symbol, price, volume insert all events into Out;",
    "length_expired_agg": "from StockStream[price > 30]#window.length(7) select symbol, sum(volume) as v, "
                          "avg(price) as a, count() as c insert expired events into Out;",
    "length_all_group": "from StockStream#window.length(6) select symbol, sum(price) as sp, count() as c "
                        "group by symbol insert all events into Out;",
    "length_having": "from StockStream#window.length(10) select symbol, sum(volume) as v group by symbol "
                     "having v > 1500 insert into Out;",
    "length_order_limit": "from StockStream#window.length(4) select symbol, price, volume order by price asc "
                          "limit 1 offset 1 insert into Out;",
    "length_zero": "from StockStream#window.length(0) select symbol, sum(volume) as v, count() as c "
                   "insert all events into Out;",
    "batch_all_events": "from StockStream#window.lengthBatch(4) select symbol, sum(price) as s, volume "
                        "insert all events into Out;",
    "batch_group_order": "from StockStream#window.lengthBatch(8) select symbol, sum(volume) as tv, price "
                         "group by symbol order by tv desc, symbol limit 3 insert into Out;",
    "batch_stream_current": "from StockStream#window.lengthBatch(3, true) select symbol, count() as c, "
                            "avg(price) as m insert all events into Out;",
    "batch_stream_group": "from StockStream#window.lengthBatch(4, true) select symbol, sum(volume) as v "
                          "group by symbol insert all events into Out;",
    "batch_offset": "from StockStream#window.lengthBatch(5) select symbol, price order by price desc offset 2 "
                    "insert into Out;",
    "batch_zero": "from StockStream#window.lengthBatch(0) select symbol, count() as c insert all events into Out;",
    "no_window_expr": "from StockStream[volume > 300] select symbol, price * 2 as p2, volume + 1 as v1, "
                      "price > 50.0 as hi insert into Out;",
    "no_window_running_agg": "from StockStream select symbol, sum(volume) as tv, volume "
                             "group by symbol, volume > 500 insert into Out;",
    "agg_expression": "from StockStream#window.length(9) select symbol, sum(volume) * 2 + count() as x, "
                      "avg(price) - 1.5 as d group by symbol insert into Out;",
    "length_minmax_all": "from StockStream#window.length(6) select symbol, min(price) as lo, max(volume) as hi "
                         "group by symbol insert all events into Out;",
    "minmax_spread": "from StockStream#window.length(9) select symbol, max(price) - min(price) as spread "
                     "group by symbol insert into Out;",
    "batch_minmax": "from StockStream#window.lengthBatch(3, true) select symbol, count() as c, "
                    "max(price) as m insert all events into Out;",
    "batch_min_nostream": "from StockStream#window.lengthBatch(4) select symbol, min(volume) as lo "
                          "insert all events into Out;",
}

PART = {
    "part_length_expired": "from StockStream#window.length(2) select symbol, sum(price) as price, volume "
                           "insert expired events into Out;",
    "part_batch_all": "from StockStream#window.lengthBatch(3) select symbol, sum(price) as price, volume "
                      "insert all events into Out;",
    "part_batch_stream": "from StockStream#window.lengthBatch(2, true) select symbol, sum(volume) as v "
                         "insert all events into Out;",
    "part_length_current": "from StockStream#window.length(4) select symbol, avg(volume) as av, count() as c "
                           "insert into Out;",
    "part_group_having": "from StockStream#window.length(5) select symbol, volume > 500 as big, count() as c "
                         "group by volume > 500 having c > 1 insert into Out;",
    "part_length_max": "from StockStream#window.length(4) select symbol, avg(volume) as av, max(price) as mp "
                       "insert into Out;",
    "part_time_current": "from StockStream#window.time(40) select symbol, sum(volume) as v, max(price) as mp "
                         "insert into Out;",
}


def _run(ql, n, k, seed, flush_every, chunk=None, sleeps=0, step_ms=7, ncols=4, playback=False):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "window", g.path("query1")
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    assert np.array_equal(oi, gi)
    d = synth.stock_ticks(n, seed=seed, k=k)
    d["ts"] = synth.T0 + np.arange(n, dtype=np.int64) * step_ms
    cols = [gi[d["symbol"]], d["price"], d["volume"]]
    raw = raw_matrix(TYPES, cols)
    si = o.L.or_stream_index(o.h, b"StockStream")
    step = chunk or 1
    rng = np.random.default_rng(seed)
    dev, sent = [], 0
    for s in range(0, n, step):
        if sleeps and rng.random() < 0.2:
            t = int(d["ts"][s]) - 1 + int(rng.integers(0, sleeps))
            o.set_time(t)
            g.set_time(t)
        o.send_columns(si, d["ts"][s:s + step], raw[s:s + step], None, chunk is not None)
        g.send_columns("StockStream", d["ts"][s:s + step], [c[s:s + step] for c in cols], chunk is not None)
        sent += step
        if sent >= flush_every:
            g.flush()
            dev.append(g.kernel_ms("gw_device"))
            sent = 0
    compare_raw(o.raw_outputs(), g.raw_outputs(), ncols)
    assert dev and all(x == 1 for x in dev), dev      # every flush ran on the device
    return g


@pytest.mark.parametrize("name", sorted(SINGLE))
@pytest.mark.parametrize("batch", [False, True])
def test_device_single_stream(name, batch):
    ql = S + " @info(name='query1') " + SINGLE[name]
    _run(ql, 2500, 6, seed=len(name), flush_every=97, chunk=13 if batch else None)


@pytest.mark.parametrize("name", sorted(PART))
@pytest.mark.parametrize("batch", [False, True])
def test_device_partitioned(name, batch):
    ql = S + " partition with (symbol of StockStream) begin @info(name='query1') " + PART[name] + " end;"
    _run(ql, 2500, 9, seed=3 + len(name), flush_every=61, chunk=17 if batch else None)


@pytest.mark.parametrize("events", ["all", "expired"])
def test_device_time_window_timer_chunks(events):
    """Clock advances between sends fire TIMER chunks that expire the due rows (expired output visible)."""
    ql = (S + " @info(name='query1') from StockStream#window.time(50) select symbol, sum(volume) as v, price "
          f"insert {events} events into Out;")
    _run(ql, 2000, 5, seed=7, flush_every=83, sleeps=120, step_ms=9)


def test_device_partitioned_time_window_ticks():
    """Partitioned time window, current events: clock advances expire rows between an instance's events; the
    aggregates its next event sees are the same whichever tick drained them."""
    ql = (S + " partition with (symbol of StockStream) begin @info(name='query1') from StockStream#window.time(60) "
          "select symbol, sum(price) as sp, count() as c, min(volume) as lo insert into Out; end;")
    _run(ql, 2500, 7, seed=17, flush_every=89, sleeps=150, step_ms=5)


def test_device_time_window_playback_group():
    ql = ("@app:playback " + S + " @info(name='query1') from StockStream#window.time(40) "
          "select symbol, count() as c, avg(price) as ap, min(price) as lo group by symbol "
          "insert all events into Out;")
    _run(ql, 2000, 5, seed=9, flush_every=101, step_ms=6)


def test_device_time_window_batches():
    ql = ("@app:playback " + S + " @info(name='query1') from StockStream#window.time(30) "
          "select symbol, sum(price) as sp insert all events into Out;")
    _run(ql, 3000, 4, seed=12, flush_every=150, chunk=25, step_ms=3)


def test_device_large_flush():
    """One large flush (200K events, 64 groups) and a second from its carried state."""
    ql = (S + " @info(name='query1') from StockStream[price > 10]#window.length(1000) "
          "select symbol, sum(volume) as v, avg(price) as a, count() as c group by symbol "
          "insert all events into Out;")
    _run(ql, 200_000, 64, seed=5, flush_every=100_000, chunk=1000)


PATTERN_SEL = {
    "sum_group": "from every e1=StockStream[price > 50] -> e2=StockStream[volume > e1.volume] "
                 "select e1.symbol, sum(e2.price) as total, count() as c group by e1.symbol insert into Out;",
    "having_order": "from every e1=StockStream[price > 60] -> e2=StockStream[price < e1.price] "
                    "select e1.symbol, e2.price as p, max(e2.volume) as mv having mv > 200 "
                    "order by p desc limit 1 insert into Out;",
    "avg_expr": "from every e1=StockStream -> e2=StockStream[symbol == e1.symbol] "
                "select e1.symbol, avg(e2.price - e1.price) * 10 as d insert into Out;",
    "min_running": "from every e1=StockStream[price > 40] -> e2=StockStream[price > e1.price] "
                   "select e1.symbol, min(e2.price) as lo, count() as c insert into Out;",
}


def _run_pattern(ql, n, k, seed, flush_every, part=False):
    o = OracleApp(ql); o.add_query_callback("query1"); o.start()
    g = GpuApp(ql); g.add_query_callback("query1"); g.start()
    assert g.path("query1") == "nfa"
    oi, gi = intern_symbols(o, k), intern_symbols(g, k)
    d = synth.stock_ticks(n, seed=seed, k=k)
    d["ts"] = synth.T0 + np.arange(n, dtype=np.int64) * 7
    cols = [gi[d["symbol"]], d["price"], d["volume"]]
    raw = raw_matrix(TYPES, cols)
    si = o.L.or_stream_index(o.h, b"StockStream")
    dev = []
    for s in range(0, n, flush_every):
        o.send_columns(si, d["ts"][s:s + flush_every], raw[s:s + flush_every], None, False)
        g.send_columns("StockStream", d["ts"][s:s + flush_every], [c[s:s + flush_every] for c in cols], False)
        g.flush()
        dev.append(g.kernel_ms("nfa_device_selector"))
    compare_raw(o.raw_outputs(), g.raw_outputs(), 3)
    ran = [x for x in dev if x >= 0]
    assert ran and all(x == 1 for x in ran), dev    # the selector stage ran on the device


@pytest.mark.parametrize("name", sorted(PATTERN_SEL))
def test_device_pattern_selector(name):
    """The NFA's selector stage (one chunk per match, StreamPostStateProcessor -> QuerySelector) on the device,
    aggregator states carried across flushes."""
    _run_pattern(S + " @info(name='query1') " + PATTERN_SEL[name], 1500, 4, seed=5 + len(name), flush_every=173)


def test_device_partitioned_pattern_selector():
    ql = (S + " partition with (symbol of StockStream) begin @info(name='query1') "
          "from every e1=StockStream[price > 40] -> e2=StockStream[price > e1.price] "
          "select e1.symbol, sum(e2.volume) as tv, min(e2.price) as lo insert into Out; end;")
    _run_pattern(ql, 3000, 7, seed=21, flush_every=211)
