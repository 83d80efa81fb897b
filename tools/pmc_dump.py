#!/usr/bin/env python3
"""Per-launch PMC counters of one kernel from rocprofv3 --pmc passes (one directory per pass, every
*counter_collection.csv below `root`), as JSON for profiles/: each counter summed over the kernel's dispatches and
divided by their number, plus the SQ wave-state fractions. FETCH_SIZE is reported as is (KiB) and doubled into
hbm_read_bytes (gfx950's streaming-read undercount, MI355X_MICROARCH.md); WRITE_SIZE (KiB) into hbm_write_bytes."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("kernel")
    ap.add_argument("-o", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    tot, disp = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    per = {k: tot[k] / max(1, len(disp[k])) for k in tot}
    out = {"kernel": a.kernel, "note": a.note, "dispatches": {k: len(v) for k, v in disp.items()},
           "per_launch": {k: round(v, 1) for k, v in sorted(per.items())}}
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        out["wave_state_fractions"] = {k: round(per[k] / wc, 4) for k in (
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
            "SQ_ACTIVE_INST_VMEM") if k in per}
    if "FETCH_SIZE" in per:
        out["hbm_read_bytes"] = round(2 * per["FETCH_SIZE"] * 1024)
    if "WRITE_SIZE" in per:
        out["hbm_write_bytes"] = round(per["WRITE_SIZE"] * 1024)
    json.dump(out, open(a.o, "w"), indent=1)
    print(json.dumps(out)[:600])


if __name__ == "__main__":
    main()
