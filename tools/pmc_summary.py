"""Per-kernel averages of rocprofv3 --pmc CSV output (tools/pmc.sh).

    python tools/pmc_summary.py gpurun_out/pmc_TAG [kernel-substring ...]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main(d, pats):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"\(.*$", "", row["Kernel_Name"])[:70]
            if pats and not any(p in k for p in pats):
                continue
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} mean {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
