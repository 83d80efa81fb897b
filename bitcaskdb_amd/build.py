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


def build(force: bool = False, verbose: bool = True, sanitize: bool = False) -> str:
    """sanitize: an ASan/UBSan build of the host code (device code unchanged) as libbcw_asan.so, for
    tools/sanitize_cpu.sh"""
    out = os.path.join(HERE, "libbcw_asan.so") if sanitize else OUT
    deps = SRCS + [os.path.join(HERE, "csrc", h) for h in ("bcw_internal.h", "bcw_parse.h")] + \
        [os.path.join(ROOT, "include", "bcw.h")]
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    san = ["-Xarch_host", "-fsanitize=address,undefined", "-Xarch_host", "-shared-libsan", "-Xarch_host",
           "-fno-omit-frame-pointer", "-g"] if sanitize else []
    cmd = ["hipcc", "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared", "-Xarch_host", "-msse4.2", *san,
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc"), *SRCS, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, sanitize="--sanitize" in sys.argv)
