"""Debug: NFA device push vs host push vs oracle, one chunk of n events (config 3 every)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..")); sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from oracle.pyoracle import OracleApp
from siddhi_amd import synth
from siddhi_amd.runtime import GpuApp
from synth_run import intern_symbols, raw_matrix
from test_gpu_nfa_configs import CONFIG3_EVERY
T = ["STRING", "FLOAT", "INT"]
for n, spec in [(20000, "0"), (20000, "1"), (60000, "0")]:
    os.environ["SG_NFA_SPEC"] = spec; os.environ["SG_NFA_SEG"] = "256"; os.environ["SG_NFA_WARM"] = "32"
    k = 40
    d = synth.stock_ticks(n, seed=synth.SEEDS[3] + 5, k=k, e=1)
    o = OracleApp(CONFIG3_EVERY); o.add_query_callback("query1"); o.start()
    gh = GpuApp(CONFIG3_EVERY); gh.add_query_callback("query1"); gh.start()
    gd = GpuApp(CONFIG3_EVERY); gd.add_query_callback("query1"); gd.start()
    oi, hi, di = intern_symbols(o, k), intern_symbols(gh, k), intern_symbols(gd, k)
    sym = di[d["symbol"]]
    raw = raw_matrix(T, [sym, d["price"], d["volume"]])
    o.send_columns(o.L.or_stream_index(o.h, b"StockStream"), d["ts"], raw, None, True)
    gh.send_columns("StockStream", d["ts"], [sym, d["price"], d["volume"]], True)
    dev = torch.device("cuda", 0)
    ts = torch.from_numpy(d["ts"]).to(dev)
    cols = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in (sym, d["price"], d["volume"])]
    torch.cuda.synchronize()
    gd.push_device("StockStream", n, ts.data_ptr(), [c.data_ptr() for c in cols], hip_stream=torch.cuda.current_stream(dev).cuda_stream, batch=True)
    oo, ho, do = o.raw_outputs(), gh.raw_outputs(), gd.raw_outputs()
    print(n, spec, "callbacks oracle", len(oo[0]["kind"]), "host", len(ho[0]["kind"]), "dev", len(do[0]["kind"]),
          "rows", len(oo[1]), len(ho[1]), len(do[1]))
    if len(do[0]["kind"]) != len(oo[0]["kind"]):
        print(" dev first seqs", do[0]["seq"][:10], "oracle ts", oo[0]["ts"][:5], "dev ts", do[0]["ts"][:5])
