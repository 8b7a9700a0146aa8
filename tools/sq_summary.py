"""Summarise rocprofv3 --pmc passes (tools/pmc.sh: one counter group per pass, kernel trace only) for one kernel.

    python tools/sq_summary.py gpurun_out/pmc_TAG KERNEL_SUBSTRING STEPS EVENTS_PER_STEP "what" > profiles/rNN_....txt

Counters are summed over every dispatch of the kernel in a pass and divided by STEPS (the bench's warm-up plus timed
steps: each step runs the same work).  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md); the shares below are ratios of those, so the unit cancels.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, kern, steps, events, what):
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if kern not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row["Dispatch_Id"])
    print(f"rocprofv3 --pmc passes ({d}), kernel *{kern}*, counters summed over its dispatches / {steps} steps;")
    print(what)
    print("SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md).")
    for k in sorted(tot):
        v = tot[k] / steps
        print(f"{k:24s} {v:.4g} per step  ({v / events:.1f} per event, {len(disp[k])} dispatches)")
    wc = tot.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print(f"share of wave cycles: parked on s_waitcnt/barrier (SQ_WAIT_ANY) {100 * tot['SQ_WAIT_ANY'] / wc:.1f}%, "
              f"issuing (SQ_ACTIVE_INST_ANY) {100 * tot['SQ_ACTIVE_INST_ANY'] / wc:.1f}%, "
              f"issue-stalled (SQ_WAIT_INST_ANY) {100 * tot['SQ_WAIT_INST_ANY'] / wc:.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else "")
