"""Deterministic synthetic StockStream ticks (BASELINE.md "Synthetic inputs").

    r_i    = splitmix64(seed + i)
    symbol = r % K                       (dictionary id of "S<id>")
    price  = (float)(1000 + (r >> 20) % 9000) / 100f      in [10.00, 99.99]
    volume = (int)((r >> 40) % 1000)
    ts_i   = T0 + floor(i / E)           (E events per millisecond, non-decreasing)
"""
import numpy as np

T0 = 1_700_000_000_000
SEEDS = {1: 0xC0FF01, 2: 0xC0FF02, 3: 0xC0FF03, 4: 0xC0FF04, 5: 0xC0FF05}


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stock_ticks(n: int, seed: int = SEEDS[1], k: int = 1000, e: int = 1, start: int = 0):
    """-> dict(ts int64, symbol int32, price float32, volume int32) for events [start, start+n)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    r = splitmix64(np.uint64(seed) + i)
    sym = (r % np.uint64(k)).astype(np.int32)
    price = (np.float32(1000) + ((r >> np.uint64(20)) % np.uint64(9000)).astype(np.float32)) / np.float32(100)
    vol = ((r >> np.uint64(40)) % np.uint64(1000)).astype(np.int32)
    ts = (np.int64(T0) + (np.arange(start, start + n, dtype=np.int64) // np.int64(e))).astype(np.int64)
    return {"ts": ts, "symbol": sym, "price": price.astype(np.float32), "volume": vol}


STOCK_STREAM = "define stream StockStream (symbol string, price float, volume int);"
CONFIG1_QL = (STOCK_STREAM + " @info(name='query1') from every e1=StockStream[price>20] -> "
              "e2=StockStream[price>e1.price] within 1 sec select e1.symbol, e2.price insert into Out;")
CONFIG2_QL = (STOCK_STREAM + " @info(name='query1') from StockStream[price>20]#window.length(1000) "
              "select symbol, avg(price) as avgPrice, sum(price) as total, count() as cnt "
              "group by symbol insert into Out;")
# BASELINE config 3 (count/Kleene sequence), `every` variant, partitioned by symbol for parallelism (§8d)
CONFIG3_QL = (STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') "
              "from every e1=StockStream, e2=StockStream[price>e1.price]+, e3=StockStream[price<e2[last].price] "
              "select e1.symbol, e1.price as p1, e2[last].price as p2, e3.price as p3 insert into Out; end;")
# BASELINE config 5, logical half (partitioned absent states are not lowered: DESIGN.md §1.1)
CONFIG5_QL = (STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') "
              "from every (e1=StockStream[price>80] and e2=StockStream[volume>900]) -> e3=StockStream[price<15] "
              "within 1 sec select e1.symbol, e1.price as p1, e2.volume as v2, e3.price as p3 insert into Out; end;")
# BASELINE config 5 in full: an upstream time window (event-time expiry in playback) feeds a partitioned
# logical + absent pattern through an inserted stream (hazard 14)
CONFIG5_FULL_QL = ("@app:playback " + STOCK_STREAM +
                   " @info(name='window') from StockStream#window.time(5 sec) "
                   "select symbol, sum(volume) as vol5 group by symbol insert into VolStream;"
                   " partition with (symbol of StockStream, symbol of VolStream) begin @info(name='query1') "
                   "from every (e1=StockStream[price > 80] and e2=StockStream[volume > 900]) -> "
                   "not VolStream[vol5 > 4500] for 5 sec "
                   "select e1.symbol, e1.price as p1, e2.volume as v2 insert into Out; end;")


def stock_ticks_rr(n: int, seed: int, k: int, start: int = 0):
    """Config-5 stream: one event per ms and round-robin keys (event i has key i mod k).  With k
    dividing the 5 s wait every key's Scheduler deadlines stay in its own residue class of event
    time, so no two partition instances share a deadline (the jittered stream of SURVEY §8d)."""
    d = stock_ticks(n, seed=seed, k=k, e=1, start=start)
    d["symbol"] = (np.arange(start, start + n, dtype=np.int64) % k).astype(np.int32)
    return d


CONFIG4_QL = (STOCK_STREAM + " partition with (symbol of StockStream) begin @info(name='query1') "
              "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
              "select e1.symbol, e2.price insert into Out; end;")


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= (1 << 63) else c


def stock_ticks_torch(n: int, seed: int, k: int, e: int, start: int = 0, device="cuda"):
    """Same stream as stock_ticks, generated on the device with int64 (two's complement) torch ops.

    Unsigned arithmetic on int64 lanes: multiplication wraps identically, logical shifts are
    arithmetic shifts masked to the surviving bits, r % k goes through the halved value.
    """
    import torch
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    z = i + _s64((seed + 0x9E3779B97F4A7C15) % (1 << 64))

    def lsr(x, s):
        return (x >> s) & ((1 << (64 - s)) - 1)

    z = (z ^ lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ lsr(z, 27)) * _s64(0x94D049BB133111EB)
    r = z ^ lsr(z, 31)
    half = lsr(r, 1)
    sym = ((half % k) * 2 + (r & 1)) % k
    price = (lsr(r, 20) % 9000 + 1000).to(torch.float32) / 100.0
    vol = lsr(r, 40) % 1000
    ts = T0 + torch.div(i, e, rounding_mode="floor")
    return {"ts": ts, "symbol": sym.to(torch.int32), "price": price.to(torch.float32), "volume": vol.to(torch.int32)}
