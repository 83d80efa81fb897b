#!/usr/bin/env python3
"""Per-kernel durations of one window of dispatches from a rocprofv3 --kernel-trace CSV: bench.py's launches are
1 gate decode per in-flight segment, --warmup, --steps timed, then untimed extras; this summarises the timed ones
(the rocprofv3 --stats average also counts the gate, the warmup -- which spans the chip's clock transient -- and the
extras)."""
import argparse
import csv
import glob
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace_dir")
ap.add_argument("--skip", type=int, required=True, help="pipelines before the timed ones (gate + warmup)")
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("-o", required=True)
a = ap.parse_args()
f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
out = {"source": os.path.basename(f), "window": {"skip": a.skip, "steps": a.steps}, "kernels": {}}
for name in ("k_chase", "k_crc"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if f"bcw::{name}<" in r["Kernel_Name"]]
    w = d[a.skip:a.skip + a.steps]
    out["kernels"][name] = {"dispatches_total": len(d), "timed_avg_us": round(statistics.mean(w), 2),
                            "timed_min_us": round(min(w), 2), "timed_max_us": round(max(w), 2),
                            "all_avg_us": round(statistics.mean(d), 2)}
starts = [int(r["Start_Timestamp"]) for r in rows if "bcw::k_chase<" in r["Kernel_Name"]]
ends = [int(r["End_Timestamp"]) for r in rows if "bcw::k_crc<" in r["Kernel_Name"]]
if len(starts) > a.skip + a.steps:
    out["timed_span_us_per_step"] = round((ends[a.skip + a.steps - 1] - starts[a.skip]) / 1000 / a.steps, 2)
json.dump(out, open(a.o, "w"), indent=1)
print(json.dumps(out))
