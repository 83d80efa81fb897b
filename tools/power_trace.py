#!/usr/bin/env python3
"""Samples GPU 0's SMU metrics (per-XCD gfx clocks, memory/SoC clocks, socket power, throttle residency counters)
as fast as amdsmi returns them, for --seconds, into a CSV; started in the background beside a workload (its own
process: amdsmi reads the driver's gpu_metrics, it creates no HIP context). Every row carries CLOCK_MONOTONIC and
CLOCK_BOOTTIME so that a rocprofv3 kernel trace of the workload can be aligned with it (tools/power_align.py).

  python3 tools/power_trace.py OUT.csv --seconds 120 --stop-file STOP &
"""
import argparse
import csv
import time

import amdsmi

FIELDS = ["current_uclk", "current_socclk", "current_socket_power", "average_socket_power", "throttle_status",
          "indep_throttle_status", "ppt_residency_acc", "socket_thm_residency_acc", "prochot_residency_acc",
          "hbm_thm_residency_acc", "accumulation_counter", "firmware_timestamp", "temperature_hotspot",
          "temperature_mem", "voltage_gfx", "energy_accumulator"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--stop-file", default=None, help="stop early once this file exists")
    args = ap.parse_args()
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[args.device]
    t_end = time.monotonic() + args.seconds
    rows = []
    import os
    n = 0
    while time.monotonic() < t_end:
        n += 1
        if args.stop_file and n % 64 == 0 and os.path.exists(args.stop_file):
            break
        mono = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        boot = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        except Exception as e:  # keep sampling; record the failure once per row
            rows.append([mono, boot, f"error: {e}"])
            time.sleep(0.01)
            continue
        g = m.get("current_gfxclks")
        gl = [v for v in (g if isinstance(g, list) else []) if isinstance(v, int)]
        rows.append([mono, boot, m.get("current_gfxclk"), min(gl) if gl else "", max(gl) if gl else "",
                     *[m.get(f) for f in FIELDS]])
    amdsmi.amdsmi_shut_down()
    with open(args.out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["mono_ns", "boot_ns", "gfxclk", "gfxclk_min", "gfxclk_max", *FIELDS])
        w.writerows(rows)
    print(f"power_trace: {len(rows)} samples in {args.seconds} s -> {args.out}", flush=True)


if __name__ == "__main__":
    main()
