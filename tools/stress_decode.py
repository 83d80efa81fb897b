#!/usr/bin/env python3
"""Repeat the device decode of one large synthetic segment and compare every run with the CPU oracle
(diagnostics for nondeterminism). Usage: stress_decode.py [MiB] [value_len] [runs] [mode]"""
import ctypes as C
import faulthandler
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402
from bitcaskdb_amd import Context  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 150
vlen = int(sys.argv[2]) if len(sys.argv) > 2 else 10
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 10
seg = O.synth(mib << 20, 0, 7, 20, 100, vlen, 0)
ref = O.decode(seg, 40, 1_700_000_000, 20, 20, 0, want_bytes=False)
print(f"{len(seg)} B, {len(ref.recs)} records, {len(ref.frags)} fragments, oracle err {ref.err_class}", flush=True)
faulthandler.dump_traceback_later(40, exit=True)
ctx = Context(0)
print('ctx ok', flush=True)
bad = 0
for i in range(runs):
    print('run', i, flush=True)
    got = ctx.decode(np.frombuffer(seg, dtype=np.uint8), 40, 1_700_000_000, 20, 20, with_frags=True)
    r = got.result
    ok_bits = got.frags["crc_ok"][:len(ref.frags)]
    nbad = int((ok_bits != ref.frags["crc_ok"]).sum())
    same = (r.err_class == ref.err_class and r.n_records == len(ref.recs) and nbad == 0)
    if not same:
        bad += 1
        idx = np.nonzero(ok_bits != ref.frags["crc_ok"])[0][:8]
        print(f"run {i}: err {r.err_class} frag {r.err_frag} n {r.n_records}; crc_ok mismatches {nbad} at {idx.tolist()}",
              [(int(ref.frags['data_off'][j]), int(ref.frags['len'][j])) for j in idx[:3]], flush=True)
print(f"{bad}/{runs} runs differ")
