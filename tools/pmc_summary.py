#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of bench.py into the per-launch HBM traffic of one kernel
(profiles/rNN_k_crc_pmc.json, read by bench.py as roofline.traffic).

Reads: one pass of the size-resolved L2->memory read requests TCC_EA0_RDREQ_{32B,64B,128B}_sum (+ TCC_EA0_RDREQ_sum
as a consistency check), bytes = 32 n32 + 64 n64 + 128 n128. rocprofv3's FETCH_SIZE counts 128 B requests through
TCC_BUBBLE, which stays 0 on gfx950, so it tallies them at 64 B (MI355X_MICROARCH.md, HBM section: "FETCH_SIZE reports
exactly 1/2 of a wide coalesced streaming read"); doubling the whole FETCH_SIZE would also double the kernel's narrow
(32/64 B) requests. Writes: WRITE_SIZE (KiB; exact for 16 B-per-lane stores per the same section).
--fetch: a FETCH_SIZE pass instead of --rdreq (legacy: doubled as a whole)."""
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
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rdreq", help="pass with TCC_EA0_RDREQ_sum / _32B_sum / _64B_sum / _128B_sum")
    ap.add_argument("--fetch", help="legacy FETCH_SIZE pass (doubled)")
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_crc")
    ap.add_argument("--seg-bytes", type=int, required=True)
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("-o", required=True)
    a = ap.parse_args()
    out = {"kernel": a.kernel}
    if a.rdreq:
        n = {c: per_dispatch(a.rdreq, a.kernel, f"TCC_EA0_RDREQ{c}_sum") for c in ("", "_32B", "_64B", "_128B")}
        ids = sorted(n[""])
        fetch = [32 * n["_32B"][i] + 64 * n["_64B"][i] + 128 * n["_128B"][i] for i in ids]
        fetch_b = statistics.median(fetch)
        med = {k or "all": statistics.median(v.values()) for k, v in n.items()}
        out["read_requests_per_launch"] = {k: round(v) for k, v in med.items()}
        out["read_request_sizes_cover_all"] = abs(med["_32B"] + med["_64B"] + med["_128B"] - med["all"]) <= 0.01 * med["all"]
        nfetch = len(ids)
        corr = "reads: 32/64/128 B L2->memory requests (TCC_EA0_RDREQ_*B_sum) x their sizes; writes: WRITE_SIZE KiB"
    else:
        fe = per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")
        fetch_b = 2 * statistics.median(fe.values()) * 1024
        nfetch = len(fe)
        corr = "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes"
    wr = per_dispatch(a.write, a.kernel, "WRITE_SIZE")
    write_b = statistics.median(wr.values()) * 1024
    spec = importlib.util.spec_from_file_location(
        "_bcw_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bitcaskdb_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    out.update({"decode_src_sha16": b.decode_src_sha16(), "seg_bytes": a.seg_bytes,
                "alg_bytes_per_launch": a.alg_bytes,
                "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
                "hbm_bytes_per_launch": round(fetch_b + write_b),
                "traffic_over_alg": round((fetch_b + write_b) / a.alg_bytes, 4),
                "dispatches": {"fetch": nfetch, "write": len(wr)}, "correction": corr})
    json.dump(out, open(a.o, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
