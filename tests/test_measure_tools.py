"""The measurement helpers behind bench.py's roofline line (CPU): tools/pmc_summary.py turns the size-resolved read
requests and WRITE_SIZE of rocprofv3 --pmc passes into HBM bytes per launch (tied to the decode sources' hash), and
tools/trace_window.py averages the timed dispatches of a rocprofv3 kernel trace of bench.py."""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


def _counter_csv(path, rows):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_summary_size_resolved(tmp_path):
    rd, wr = str(tmp_path / "rd"), str(tmp_path / "wr")
    rows = []
    for d in (1, 2, 3):  # three k_crc dispatches and an unrelated kernel
        for name, v in (("TCC_EA0_RDREQ_sum", 1000 + 10), ("TCC_EA0_RDREQ_32B_sum", 0),
                        ("TCC_EA0_RDREQ_64B_sum", 10), ("TCC_EA0_RDREQ_128B_sum", 1000)):
            rows.append(dict(Dispatch_Id=d, Kernel_Name="void bcw::k_crc<0>(...)", Counter_Name=name, Counter_Value=v))
        rows.append(dict(Dispatch_Id=d + 10, Kernel_Name="other", Counter_Name="TCC_EA0_RDREQ_128B_sum",
                         Counter_Value=99999))
    _counter_csv(rd, rows)
    _counter_csv(wr, [dict(Dispatch_Id=d, Kernel_Name="void bcw::k_crc<0>(...)", Counter_Name="WRITE_SIZE",
                           Counter_Value=2.0) for d in (1, 2, 3)])
    out = str(tmp_path / "pmc.json")
    subprocess.run([sys.executable, os.path.join(TOOLS, "pmc_summary.py"), "--rdreq", rd, "--write", wr,
                    "--seg-bytes", "1000", "--alg-bytes", "100000", "-o", out], check=True, capture_output=True)
    j = json.load(open(out))
    assert j["fetch_bytes_per_launch"] == 1000 * 128 + 10 * 64
    assert j["write_bytes_per_launch"] == 2048
    assert j["hbm_bytes_per_launch"] == 1000 * 128 + 10 * 64 + 2048
    assert j["read_request_sizes_cover_all"] is True
    sys.path.insert(0, ROOT)
    from bitcaskdb_amd.build import decode_src_sha16
    assert j["decode_src_sha16"] == decode_src_sha16()


def test_trace_window(tmp_path):
    d = tmp_path / "trace"
    d.mkdir()
    rows, t = [], 0
    durs = [300, 300, 250, 210, 212, 208, 500]  # gate, warmup x2, timed x3, extra
    for i, du in enumerate(durs):
        rows.append(dict(Kernel_Name="void bcw::k_chase<0>(...)", Start_Timestamp=t, End_Timestamp=t + 20000))
        t += 20000
        rows.append(dict(Kernel_Name="void bcw::k_crc<0>(...)", Start_Timestamp=t, End_Timestamp=t + du * 1000))
        t += du * 1000
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for r in rows:
            w.writerow(r)
    out = str(tmp_path / "w.json")
    subprocess.run([sys.executable, os.path.join(TOOLS, "trace_window.py"), str(d), "--skip", "3", "--steps", "3",
                    "-o", out], check=True, capture_output=True)
    j = json.load(open(out))
    assert j["kernels"]["k_crc"]["timed_avg_us"] == 210.0
    assert j["kernels"]["k_chase"]["timed_avg_us"] == 20.0
    assert j["timed_span_us_per_step"] == (60 + 630) / 3
