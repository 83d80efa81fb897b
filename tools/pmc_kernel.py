#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters of one kernel over its dispatches (all counter_collection.csv files
under a directory) and print them with the derived wave-state fractions."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    path, kernel = sys.argv[1], sys.argv[2]
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
    print(f"{kernel}: {len(disp)} dispatches")
    for k in sorted(tot):
        print(f"  {k:28s} {tot[k]:.4g}")
    wc = tot.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if k in tot:
                print(f"  {k + ' / WAVE_CYCLES':40s} {tot[k] / wc:.3f}")


if __name__ == "__main__":
    main()
