#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into the per-launch HBM
traffic of one kernel (profiles/rNN_k_crc_pmc.json, read by bench.py as roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so it is doubled; WRITE_SIZE is taken as is. Both are in KiB."""
import argparse
import csv
import glob
import json
import os
import importlib.util
import statistics


def per_dispatch(path, kernel, counter):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_crc")
    ap.add_argument("--seg-bytes", type=int, required=True)
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("-o", required=True)
    a = ap.parse_args()
    fe = per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")
    wr = per_dispatch(a.write, a.kernel, "WRITE_SIZE")
    fetch_b = 2 * statistics.median(fe) * 1024
    write_b = statistics.median(wr) * 1024
    spec = importlib.util.spec_from_file_location(
        "_bcw_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitcaskdb_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    out = {"kernel": a.kernel, "decode_src_sha16": b.decode_src_sha16(), "seg_bytes": a.seg_bytes,
           "alg_bytes_per_launch": a.alg_bytes,
           "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
           "hbm_bytes_per_launch": round(fetch_b + write_b),
           "traffic_over_alg": round((fetch_b + write_b) / a.alg_bytes, 4),
           "dispatches": {"fetch": len(fe), "write": len(wr)},
           "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes"}
    json.dump(out, open(a.o, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
