"""HBM traffic per step of a bench workload from rocprofv3 PMC passes (tools/gpu_run.sh: FETCH_SIZE and
WRITE_SIZE in separate runs), corrected per access width.

/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE reports 1/2 of the bytes of a 16-B-per-lane streaming
read on gfx950, WRITE_SIZE is exact for 16-B stores, and other widths are uncalibrated ("calibrate on a known
byte count in your own access pattern").  tools/micro/pmc_calib.hip moves exactly 1 GiB per kernel with 4-,
8-, 12- and 16-B lanes; its PMC passes give a factor (true bytes / counter bytes) per width and direction.
Each pipeline kernel's counters are scaled by the factor of the width its bytes mostly move at (WIDTHS below:
read width, write width, from the kernels' code).  Without a calibration run the guide's rule applies to
16-B kernels only (x2 fetch) and every other width is reported unscaled.

    python tools/pmc_traffic.py gpurun_out/pmc_TAG_c4 EVENTS [gpurun_out/pmc_TAG_calib [CONFIG [RUNS]]] > profiles/rNN_keyed_traffic.json
(RUNS: the bench runs the pass profiled -- warm-up plus steps -- for kernels launched several times per step)
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

# kernel name prefix -> (read width, write width) in bytes per lane (the width carrying most of its bytes)
WIDTHS = {
    "k_kc_sort": (4, 16),      # ts / symbol / price columns (4-B and 8-B lanes), sorted chunk stored as 16-B entry pairs
    "k_kc_slices": (8, 4),
    "k_kc_match": (8, 16),     # 8-B entries gathered per chunk run, 16-B records
    "k_kt_hist": (16, 4),      # 16-B symbol loads (4 keys per lane), per-tile counts
    "k_kt_scatter": (4, 4),    # ts / symbol / price columns (8 + 4 + 4 B per event: 4-B and 8-B lanes), 12-B entries staged through LDS and stored as words
    "k_kt_tdesc": (4, 8),
    "k_kt_match": (12, 16),    # 12-B entries (KtE12), 16-B records
    "k_kt_order": (16, 16),    # 16-B records in, 16-B records out
    "k_nfa_": (4, 4),          # lane interpreter: word loads and stores
    "k_fb_tile": (8, 4),       # config 1: ts (8-B lanes) and price staged, record words (j, projections) stored
    "k_fb_list": (4, 4),
    "k_wa_filter": (4, 4),     # config 2: price words in, one flag byte per event out (word stores of 4 flags)
    "k_wa_place": (16, 4),     # 16 flags per 16-B load, event indices out
    "k_wa_gather": (4, 4),     # filtered-order columns gathered word by word
    "k_wa_wstart": (4, 4),
    "k_wa_tile": (4, 8),       # gathered words in, avg / sum / count (8-B) out
    "rocprim": (4, 4),
}
PIPE = tuple(WIDTHS)
CAL_BYTES = {4: 1 << 30, 8: 1 << 30, 12: (((1 << 30) // 12) * 12), 16: 1 << 30}


def counters(d):
    """kernel -> counter -> [per-dispatch values] over every counter_collection.csv under d"""
    per = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"\(.*$", "", row["Kernel_Name"]).replace("void ", "").replace("sg::", "")
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def cal_width(k):
    """access width of a calibration kernel from its (demangled) name"""
    if "U2" in k:
        return 8
    if "U3" in k:
        return 12
    if "vector" in k or "uint4" in k:
        return 16
    return 4


def calibration(d):
    """width -> (read factor, write factor): true bytes / counter bytes (counters are in KB)"""
    if not d or not os.path.isdir(d):
        return None
    per = counters(d)
    got = defaultdict(dict)
    for k, cs in per.items():
        for pre, ctr in (("k_rd<", "FETCH_SIZE"), ("k_wr<", "WRITE_SIZE")):
            if k.startswith(pre) and cs.get(ctr):
                got[cal_width(k)][ctr] = sum(cs[ctr]) / len(cs[ctr]) * 1024
    cal = {}
    for w in (4, 8, 12, 16):
        rd, wr = got[w].get("FETCH_SIZE"), got[w].get("WRITE_SIZE")
        cal[w] = (CAL_BYTES[w] / rd if rd else None, CAL_BYTES[w] / wr if wr else None)
    return cal


def main(d, events, cal_dir=None, config=4, runs=0):
    """runs > 0: a kernel's bytes per step are the sum over its dispatches / runs (kernels launched several times per
    step: the NFA's speculative, key and repair launches); runs = 0: the average dispatch (one launch per step)."""
    cal = calibration(cal_dir)
    per = counters(d)
    kern = {}
    tot_r = tot_w = raw_r = raw_w = 0.0
    for k, cs in per.items():
        hit = [p for p in PIPE if p in k]
        if not hit:
            continue
        rw, ww = WIDTHS[hit[0]]
        def per_step(ctr):
            v = cs.get(ctr, [0])
            return 1024 * sum(v) / (runs if runs > 0 else max(1, len(v)))
        fr_raw = per_step("FETCH_SIZE")
        wr_raw = per_step("WRITE_SIZE")
        if cal:
            f_r = cal[rw][0] or 1.0
            f_w = cal[ww][1] or 1.0
        else:
            f_r, f_w = (2.0 if rw == 16 else 1.0), 1.0
        kern[k[:80]] = {"read_bytes": fr_raw * f_r, "write_bytes": wr_raw * f_w, "read_counter_bytes": fr_raw,
                        "write_counter_bytes": wr_raw, "read_width": rw, "write_width": ww,
                        "read_factor": f_r, "write_factor": f_w}
        tot_r += fr_raw * f_r
        tot_w += wr_raw * f_w
        raw_r += fr_raw
        raw_w += wr_raw
    print(json.dumps({"config": config, "events": events, "traffic_bytes_per_step": tot_r + tot_w,
                      "read_bytes": tot_r, "write_bytes": tot_w,
                      "counter_bytes_per_step": raw_r + raw_w, "per_kernel": kern,
                      "calibration": {str(w): {"read_factor": v[0], "write_factor": v[1]} for w, v in cal.items()}
                      if cal else None,
                      "source": {"pmc": d, "calibration": cal_dir},
                      "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (per dispatch mean); "
                                "counter bytes scaled per kernel by the factor of its dominant access width, "
                                "measured on tools/micro/pmc_calib.hip (1 GiB per width) in the same session"},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None,
         int(sys.argv[4]) if len(sys.argv) > 4 else 4, int(sys.argv[5]) if len(sys.argv) > 5 else 0)
