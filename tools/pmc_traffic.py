"""HBM traffic per step of the keyed pipeline from rocprofv3 PMC passes (tools/pmc.sh), corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KB) is read from TCC_EA0_RDREQ x 64 B
and reports 1/2 of a wide streaming read on gfx950 -> x2; WRITE_SIZE (KB) is exact for 16-B stores.

    python tools/pmc_traffic.py gpurun_out/pmc_TAG EVENTS > profiles/rNN_keyed_traffic.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PIPE = ("k_kt_", "rocprim")   # the keyed pipeline's kernels (data generation is torch, outside the step)


def main(d, events):
    per = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"\(.*$", "", row["Kernel_Name"])
            if not any(p in k for p in PIPE):
                continue
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    kern = {}
    tot_r = tot_w = 0.0
    for k, cs in per.items():
        # per dispatch mean; the pipeline launches each kernel once per step (rocprim: scan kernels)
        fr = 2 * 1024 * (sum(cs.get("FETCH_SIZE", [0])) / max(1, len(cs.get("FETCH_SIZE", [0]))))
        wr = 1024 * (sum(cs.get("WRITE_SIZE", [0])) / max(1, len(cs.get("WRITE_SIZE", [0]))))
        kern[k[:80]] = {"read_bytes": fr, "write_bytes": wr}
        tot_r += fr
        tot_w += wr
    print(json.dumps({"config": 4, "events": events, "traffic_bytes_per_step": tot_r + tot_w,
                      "read_bytes": tot_r, "write_bytes": tot_w, "per_kernel": kern,
                      "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH x2 (gfx950)"},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
