"""Builds libbcw.so in-tree for gfx950 (hipcc). Used by __graft_entry__.build() and the Makefile."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("bcw_api.cpp", "bcw_decode.hip", "bcw_encode.hip", "bcw_fanout.cpp", "bcw_index.hip", "bcw_io.cpp", "bcw_read.hip")]
OUT = os.path.join(HERE, "libbcw.so")
ARCH = os.environ.get("BCW_OFFLOAD_ARCH", "gfx950")


DECODE_SRCS = [os.path.join(HERE, "csrc", f) for f in ("bcw_decode.hip", "bcw_internal.h", "bcw_parse.h")] + \
    [os.path.join(ROOT, "include", "bcw.h")]


def decode_src_sha16() -> str:
    """content hash of the decode kernels' sources: ties a committed PMC summary (profiles/rNN_k_crc_pmc.json) to the
    k_crc build it was measured on (bench.py reports roofline.traffic only when they match)"""
    import hashlib
    h = hashlib.sha256()
    for f in DECODE_SRCS:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


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
    flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Xarch_host", "-msse4.2", *san,
             "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc")]
    objdir = os.path.join(HERE, "_obj" + ("_asan" if sanitize else ""))
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in SRCS]

    def compile_one(i):  # one hipcc per source, in parallel (the codec's kernels dominate the build time)
        cmd = ["hipcc", *flags, "-c", SRCS[i], "-o", objs[i]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)

    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(SRCS), os.cpu_count() or 1)) as ex:
        list(ex.map(compile_one, range(len(SRCS))))
    subprocess.run(["hipcc", f"--offload-arch={ARCH}", "-shared", *san, *objs, "-o", out + ".tmp"], check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, sanitize="--sanitize" in sys.argv)
