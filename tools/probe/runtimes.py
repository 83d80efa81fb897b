"""Probe: two processes on one GPU, each with torch's HIP runtime and libbcw's (/opt/rocm) runtime live.
mode torch_first: torch allocates on the GPU, then bcw_ctx_create; mode bcw_first: the reverse."""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(mode):
    from bitcaskdb_amd import _lib as L
    import torch
    h = C.c_void_p()
    out = []
    if mode == "bcw_first":
        out.append(("ctx", L.lib.bcw_ctx_create(0, C.byref(h))))
    torch.cuda.set_device(0)
    x = torch.empty(1 << 20, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    out.append(("torch", float(x.sum())))
    if mode == "torch_first":
        out.append(("ctx", L.lib.bcw_ctx_create(0, C.byref(h))))
    print(mode, os.getpid(), out, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        child(sys.argv[2])
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for mode in ("torch_first", "bcw_first"):
        ps = [subprocess.Popen([sys.executable, __file__, str(n), mode]) for _ in range(n)]
        print(mode, [p.wait(timeout=120) for p in ps], flush=True)
        time.sleep(1)
