"""CPU tests of the index oracle (tests only): murmur3 Sum64 (spaolacci/murmur3 v1.1.0, the hash of
IndexOperator.Hash index.go:15-19) against its published known answers and an independent Python
restatement; Get/Put/Delete/SoftDelete semantics (index.go:81-165) and doFilter (compaction.go:329-348)
against a Python model; the recovery / compaction callback loops over decoded segments."""
from __future__ import annotations

import random

import numpy as np

import _oracle as O
import cases
from golden import pyref

# spaolacci/murmur3 murmur3_test.go known answers (seed 0): (string, h1 = Sum64, h2)
KAT = [
    (b"", 0x0000000000000000, 0x0000000000000000),
    (b"hello", 0xcbd8a7b341bd9b02, 0x5b1e906a48ae1d19),
    (b"hello, world", 0x342fac623a5ebc8e, 0x4cdcbc079642414d),
    (b"19 Jan 2038 at 3:14:07 AM", 0xb89e5988b737affc, 0x664fc2950231b2cb),
    (b"The quick brown fox jumps over the lazy dog.", 0xcd99481f9ee902c9, 0x695da1a38987b6e7),
]


def test_murmur3_known_answers():
    for s, h1, h2 in KAT:
        assert O.murmur3_128(s) == (h1, h2), s
        assert O.murmur3_sum64(s) == h1
        assert pyref.murmur3_x64_128(s) == (h1, h2), s
    # MurmurHash3_x64_128("The quick brown fox jumps over the lazy dog") = 6c1b07bc7bbc4be347939ac4a93c437a
    h1, h2 = O.murmur3_128(b"The quick brown fox jumps over the lazy dog")
    assert (h1.to_bytes(8, "little") + h2.to_bytes(8, "little")).hex() == "6c1b07bc7bbc4be347939ac4a93c437a"


def test_murmur3_vs_pyref_all_tail_lengths():
    rng = random.Random(1)
    for n in list(range(0, 70)) + [120, 127, 128, 129, 1000]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.murmur3_sum64(b) == pyref.murmur3_sum64(b), n


def test_index_semantics_vs_model():
    rng = random.Random(2)
    x, m = O.Index(), pyref.PyIndex()
    keys = [(bytes([65 + i % 3]) * 20, b"k%d" % i) for i in range(300)]
    for step in range(6000):
        ns, k = rng.choice(keys)
        op = rng.choice([0, 0, 0, 1, 2])
        fid, off, size = rng.randrange(1, 9), rng.randrange(0, 1 << 40), rng.randrange(0, 1 << 20)
        x.set(ns, k, op, fid, off, size)
        if op == 0:
            m.put(ns, k, fid, off, size)
        elif op == 1:
            m.delete(ns, k)
        else:
            m.soft_delete(ns, k)
        if step % 7 == 0:
            ns, k = rng.choice(keys)
            st, v = x.get(ns, k)
            mst, mv = m.get(ns, k)
            assert st == mst and (st == 1 or v == mv)
            src_fid, src_off = (mv[0], mv[1]) if mv and rng.random() < 0.5 else (1, 12345)
            assert bool(O.lib.oc_do_filter(x.h, ns, len(ns), k, len(k), src_fid, src_off)) == \
                m.do_filter(ns, k, src_fid, src_off)
    assert x.live() == len(m.m)


def _ns_key(r, ns=20):
    p = r["payload"]
    return p[1:1 + ns], p[r["hdr_size"]:r["hdr_size"] + r["key_len"]]


def test_recovery_and_filter_loops():
    """recoverFromWal's Put loops (db_impl.go:290-313) in ascending fid order, then compactOneWal's
    doFilter (compaction.go:299-303) of the oldest WAL: live records are kept, overwritten ones dropped."""
    rng = random.Random(3)
    wals = []
    for fid in range(1, 4):
        payloads = [cases.rec(rng.randrange(0, 400), vlen=rng.choice([10, 300, 5000])) for _ in range(300)]
        data, _ = cases.wal_of(payloads)
        wals.append(data)
    x = O.Index()
    model = pyref.PyIndex()
    for fid, data in enumerate(wals, 1):
        ec, n = x.put_segment(data, 40, cases.BASE, 20, 20, 0, fid)
        assert ec == 0 and n == 300
        for r in pyref.iterate(data, 40, cases.BASE, 20, 20)["recs"]:
            model.put(*_ns_key(r), fid, r["foff"] - 7, r["size"])
    assert x.live() == len(model.m)
    keep, nv = x.compact_filter(wals[0], 40, cases.BASE, 20, 20, 1, 300)
    assert nv == 300
    want = [0 if model.do_filter(*_ns_key(r), 1, r["foff"] - 7) else 1
            for r in pyref.iterate(wals[0], 40, cases.BASE, 20, 20)["recs"]]
    assert keep.tolist() == want and 0 < sum(want) < 300
    # the hint path gives the same index
    y = O.Index()
    for fid, data in enumerate(wals, 1):
        ec, _, _, hint = O.hint_by_wal(data, fid, 40, cases.BASE, 20, 20)
        assert y.put_segment(hint, 40, cases.BASE, 20, 0, 1, fid) == (0, 300)
    keep2, _ = y.compact_filter(wals[0], 40, cases.BASE, 20, 20, 1, 300)
    np.testing.assert_array_equal(keep, keep2)
