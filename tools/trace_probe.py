#!/usr/bin/env python3
"""Why does bench.py's timed region run k_crc slower than kbench? Decodes config B back to back with the segment in
torch memory (alloc=torch) or hipMalloc memory (alloc=hip), then a torch reduction + host pause, then again.
Run under rocprofv3 --kernel-trace and read the per-dispatch durations."""
import ctypes as C
import sys
import time

import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from bitcaskdb_amd import _lib as L  # noqa: E402
from bitcaskdb_amd import Context  # noqa: E402

alloc = sys.argv[1] if len(sys.argv) > 1 else "torch"
n_rep = int(sys.argv[2]) if len(sys.argv) > 2 else 30
BASE = 1700000000
n, r = C.c_uint64(), C.c_uint64()
assert L.lib.bcw_synth_segment(1 << 30, 0, 42, 20, 100, 4096, 0, BASE, None, 0, C.byref(n), C.byref(r)) == 0
host = torch.empty(n.value, dtype=torch.uint8).pin_memory()
assert L.lib.bcw_synth_segment(1 << 30, 0, 42, 20, 100, 4096, 0, BASE, C.c_void_p(host.data_ptr()), n.value,
                               C.byref(n), C.byref(r)) == 0
dev = torch.device("cuda", 0)
hip = C.CDLL("libamdhip64.so")
if alloc == "hip":
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n.value)) == 0
    assert hip.hipMemcpy(p, C.c_void_p(host.data_ptr()), C.c_size_t(n.value), 1) == 0  # H2D
    seg_ptr = p.value
else:
    d_seg = host.to(dev)
    seg_ptr = d_seg.data_ptr()
cap = r.value + 64
ptr_t = {"u8": L.u64p, "u4": L.u32p, "u1": L.u8p}
cols = {}
for name, dt in L.TABLE_COLUMNS:
    cols[name] = torch.empty(cap, dtype={"u8": torch.int64, "u4": torch.int32, "u1": torch.uint8}[dt], device=dev)
table = L.RecordTable(cap, *[C.cast(C.c_void_p(cols[name].data_ptr()), ptr_t[dt]) for name, dt in L.TABLE_COLUMNS])
d_res = torch.zeros(C.sizeof(L.DecodeResult), dtype=torch.uint8, device=dev)
params = L.DecodeParams(n.value, BASE, 40, 20, 20, L.MODE_RECORD)
ctx = Context(0)
stream = torch.cuda.Stream()
ctx.set_stream(stream.cuda_stream)
torch.cuda.synchronize()


def mark(tag):  # host clocks for aligning the kernel trace with tools/power_trace.py's samples
    print(f"mark {tag} mono_ns {time.clock_gettime_ns(time.CLOCK_MONOTONIC)} "
          f"boot_ns {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}", flush=True)


def run(k):
    mark("run_start")
    for _ in range(k):
        assert L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(seg_ptr), C.byref(params), C.byref(table),
                                              C.c_void_p(d_res.data_ptr())) == 0
    torch.cuda.synchronize()
    mark("run_end")


run(n_rep)
s = int((cols["status"][: r.value] != 0).sum().item())  # a torch reduction, as bench.py's correctness gate
time.sleep(0.2)
run(n_rep)
print("done", alloc, s)
