"""Times one process's compaction fan-out (bcw_compact_wals, doCompactionWork's loop compaction.go:201-211 over
compactOneWal + doFilter) of 4 x 1 GiB config-B sources on 1 and 2 contexts of device 0, against the serial loop of
bcw_compact_segment calls. Every source's rows are live in the index (recovered first), so every row is kept and the
outputs are ~4.3 GB of dst WAL and ~0.15 GB of hint WAL, copied to preallocated host buffers. The call, not the
Python wrapper, is timed. Prints one JSON line."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bitcaskdb_amd import _lib as L  # noqa: E402
from bitcaskdb_amd import index as IX  # noqa: E402
from bitcaskdb_amd.wal import Context  # noqa: E402

BASE = 1_700_000_000


def synth(seed: int):
    n, r = C.c_uint64(), C.c_uint64()
    assert L.lib.bcw_synth_segment(1 << 30, 0, seed, 20, 100, 4096, 0, BASE, None, 0, C.byref(n), C.byref(r)) == 0
    h = np.empty(n.value, dtype=np.uint8)
    assert L.lib.bcw_synth_segment(1 << 30, 0, seed, 20, 100, 4096, 0, BASE, C.c_void_p(h.ctypes.data), n.value,
                                   C.byref(n), C.byref(r)) == 0
    return h, int(r.value)


def main():
    nsrc = int(os.environ.get("FANOUT_SOURCES", "4"))
    srcs = [synth(42 + k) for k in range(nsrc)]
    ctx, ctx2 = Context(0), Context(0)
    ix = IX.Index(ctx, keys=1 << 21, arena_bytes=256 << 20)
    for k, (data, _) in enumerate(srcs):
        ix.recover_segment(data, L.MODE_RECORD, k + 1, 40, BASE, 20, 20)
    outs = []
    arr = (L.CompactSrc * nsrc)()
    for k, (data, nrec) in enumerate(srcs):
        m = data.size
        wal = np.empty(m + m // 8 + 4096, dtype=np.uint8)
        hb = np.empty(m // 16 + 4096, dtype=np.uint8)
        offs = np.empty(nrec + 16, dtype=np.uint64)
        wal[::4096] = 0  # (touch the pages once: the first pass must not time page faults)
        hb[::4096] = 0
        outs.append((wal, hb, offs))
        arr[k].fid = k + 1
        arr[k].data = data.ctypes.data
        arr[k].len = m
        arr[k].start_off = 40
        arr[k].out = L.EncodeOut(wal.ctypes.data_as(L.u8p), wal.size, hb.ctypes.data_as(L.u8p), hb.size,
                                 offs.ctypes.data_as(L.u64p), offs.size)
    p = L.EncodeParams(0, BASE, 99, 40, 40, 0, L.ENC_COMPACT, 20, 20)
    res = (L.EncodeResult * nsrc)()
    filt = (L.IndexResult * nsrc)()

    def fan(contexts):
        ctxs = (C.c_void_p * len(contexts))(*[c.handle for c in contexts])
        done = C.c_uint64(0)
        t0 = time.perf_counter()
        rc = L.lib.bcw_compact_wals(ix.handle, ctxs, len(contexts), arr, nsrc, C.byref(p), res, filt, C.byref(done))
        dt = time.perf_counter() - t0
        assert rc == 0 and done.value == nsrc, (rc, done.value)
        assert all(res[k].err_class == 0 and res[k].n_written == srcs[k][1] for k in range(nsrc))
        return dt

    def serial():
        t0 = time.perf_counter()
        wp, hp = 40, 40
        for k in range(nsrc):
            q = L.EncodeParams(arr[k].len, BASE, 99, wp, hp, 40, L.ENC_COMPACT, 20, 20)
            r, f = L.EncodeResult(), L.IndexResult()
            rc = L.lib.bcw_compact_segment(ctx.handle, ix.handle, C.c_void_p(arr[k].data), C.byref(q), k + 1,
                                           C.byref(arr[k].out), C.byref(r), C.byref(f))
            assert rc == 0 and r.err_class == 0 and r.n_written == srcs[k][1]
            wp, hp = r.wal_end, r.hint_end
        return time.perf_counter() - t0

    fan([ctx])  # warm: scratch and pinned staging of both contexts
    fan([ctx, ctx2])
    serial()
    def snap(on):
        for c in (ctx, ctx2):
            c.set_option(L.OPT_FILTER_SNAPSHOT, int(on))

    snap(True)
    fan([ctx, ctx2])  # (warm the staging indexes)
    snap(False)
    t = {"serial_compact_segment": [], "fanout_1ctx": [], "fanout_2ctx": [], "fanout_2ctx_snapshot": []}
    for _ in range(3):
        t["serial_compact_segment"].append(serial())
        t["fanout_1ctx"].append(fan([ctx]))
        t["fanout_2ctx"].append(fan([ctx, ctx2]))
        snap(True)
        t["fanout_2ctx_snapshot"].append(fan([ctx, ctx2]))
        snap(False)
    src_bytes = sum(int(d.size) for d, _ in srcs)
    line = {"what": "bcw_compact_wals: %d x 1 GiB config-B sources, all rows kept, outputs to host" % nsrc,
            "src_bytes": src_bytes,
            "wal_bytes": int(sum(res[k].wal_need for k in range(nsrc))),
            "seconds_median": {k: round(sorted(v)[1], 4) for k, v in t.items()},
            "GiBs_median": {k: round(src_bytes / 2**30 / sorted(v)[1], 2) for k, v in t.items()},
            "runs": {k: [round(x, 4) for x in v] for k, v in t.items()}}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
