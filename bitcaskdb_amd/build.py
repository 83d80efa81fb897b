"""Builds libbcw.so in-tree for gfx950 (hipcc). Used by __graft_entry__.build() and the Makefile."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("bcw_api.cpp", "bcw_decode.hip", "bcw_encode.hip", "bcw_index.hip", "bcw_io.cpp", "bcw_read.hip")]
OUT = os.path.join(HERE, "libbcw.so")
ARCH = os.environ.get("BCW_OFFLOAD_ARCH", "gfx950")


def build(force: bool = False, verbose: bool = True) -> str:
    deps = SRCS + [os.path.join(HERE, "csrc", h) for h in ("bcw_internal.h", "bcw_parse.h")] + \
        [os.path.join(ROOT, "include", "bcw.h")]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        return OUT
    cmd = ["hipcc", "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared", "-Xarch_host", "-msse4.2",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc"), *SRCS, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
