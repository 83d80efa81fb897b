"""CPU tests of the parity oracle: known answers, golden fixtures, and cross-checks against the
independent pure-Python restatement (tests/golden/pyref.py)."""
from __future__ import annotations

import glob
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

import _oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import pyref as P  # noqa: E402

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "*.json")))


def test_crc_known_answers():
    assert O.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    assert O.compute_crc32(b"123456789") == 0xC78AB0E5
    assert O.compute_crc32(b"") == 0xA282EAD8  # empty fragment: an all-zero header fails CRC
    assert P.crc32c_bitwise(b"123456789") == 0xE3069283
    assert P.compute_crc32(b"") == 0xA282EAD8


@pytest.mark.parametrize("n", [0, 1, 3, 7, 8, 100, 4095, 4096, 12287, 12288, 12289, 40000])
def test_crc_hw_matches_table(n):
    data = bytes(random.Random(n).getrandbits(8) for _ in range(n))
    assert O.crc32c_hw(data) == O.crc32c(data)
    if n <= 4096:
        assert O.crc32c(data) == P.crc32c_bitwise(data)


def test_uvarint_go_semantics():
    cases = [b"", b"\x00", b"\x7f", b"\x80\x01", b"\xff\x7f", b"\x80", b"\x80\x80\x80",
             b"\xff" * 9 + b"\x01", b"\xff" * 9 + b"\x02", b"\xff" * 10 + b"\x00", b"\x80" * 11]
    for c in cases:
        assert O.uvarint(c) == P.go_uvarint(c), c
    for v in [0, 1, 127, 128, 300, 4096, 2 ** 32, 2 ** 63, 2 ** 64 - 1]:
        assert O.put_uvarint(v) == P.put_uvarint(v)
        assert O.uvarint(O.put_uvarint(v)) == (v, len(P.put_uvarint(v)))


def _rand_record(rng, base):
    ns = bytes(rng.getrandbits(8) for _ in range(20))
    key = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 200)))
    val = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 100, 4096, 33000, 70000])))
    etag = bytes(rng.getrandbits(8) for _ in range(20)) if rng.random() < 0.5 else b""
    expire = 0 if rng.random() < 0.5 else base + rng.randrange(0, 1 << 34)
    meta = b"\x81\xa1k\xa1v" if rng.random() < 0.3 else b""
    return ns, key, val, etag, expire, rng.random() < 0.3, meta


@pytest.mark.parametrize("seed", range(6))
def test_record_encode_parity(seed):
    rng = random.Random(seed)
    base = 1_700_000_000
    for _ in range(30):
        ns, key, val, etag, expire, tomb, meta = _rand_record(rng, base)
        a = O.record_encode(ns, key, val, etag, expire, tomb, meta, base)
        b = P.record_encode(ns, key, val, etag, expire, tomb, meta, base)
        assert a == b
        if a is None:  # expire delta >= 2^35: the reference panics (both restatements agree)
            continue
        st, f = P.record_from_bytes(a, base, 20, 20)
        assert st == 0 and f["key_len"] == len(key) and f["val_len"] == len(val)
    assert O.record_encode(b"", b"k", b"v", b"", base - 1, False, b"", base) is None  # "invalid expire"


@pytest.mark.parametrize("seed", range(4))
def test_writer_parity_with_pyref(seed):
    rng = random.Random(100 + seed)
    w, pw = O.Writer(5, 7), P.PyWal(5, 7)
    for _ in range(40):
        n = rng.choice([1, 2, 7, 100, 4222, 32754, 32761, 32762, 40000, 70000])
        rec = bytes(rng.getrandbits(8) for _ in range(n))
        assert w.write(rec) == pw.write_record(rec)
    assert w.data() == bytes(pw.buf)


def test_writer_branches():
    """padding (leftover < 7) and zero-length First (leftover == 7) are produced."""
    w = O.Writer(0, 0)
    w.write(bytes(32768 - 7 - 3))
    off = w.write(b"x" * 100)
    assert off == 40 + 32768  # 3 padding bytes skipped
    w2 = O.Writer(0, 0)
    w2.write(bytes(32768 - 7 - 7))
    off2 = w2.write(b"y" * 100)
    data = w2.data()
    assert off2 == 40 + 32768 - 7
    assert data[off2 + 4:off2 + 7] == b"\x00\x00\x02"  # zero-length First
    d = O.decode(data, 40, 0, 20, 20)
    assert d.recs["foff"][-1] == 40 + 32768 + 7  # iterator re-captures the offset (quirk 8.2.1)


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-5] for p in GOLDEN])
def test_oracle_matches_golden(path):
    exp = json.load(open(path))
    data = open(path[:-5] + ".wal", "rb").read()
    assert hashlib.sha1(data).hexdigest() == exp["file_sha1"]
    p = exp["params"]
    d = O.decode(data, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"])
    assert d.err_class == exp["err_class"]
    if exp["err_frag"] is not None:
        assert d.err_frag == exp["err_frag"]
    assert len(d.frags) == len(exp["frags"])
    for got, want in zip(d.frags, exp["frags"]):
        for k in ("data_off", "len", "stored_crc", "type", "crc_ok"):
            assert int(got[k]) == want[k], k
    assert len(d.recs) == len(exp["recs"])
    for i, (got, want) in enumerate(zip(d.recs, exp["recs"])):
        for k in ("foff", "size", "first_frag", "emit_frag", "status", "hdr_size", "key_len"):
            assert int(got[k]) == want[k], (i, k)
        if p["mode"] == 0:
            for k in ("flags", "etag_off", "val_len", "meta_len", "expire"):
                assert int(got[k]) == want[k], (i, k)
        else:
            assert int(got["expire"]) == want["fid"]
            assert int(got["val_len"]) == want["off"]
            assert int(got["meta_len"]) == want["hint_size"]
        assert hashlib.sha1(d.payloads[i]).hexdigest() == want["payload_sha1"]


@pytest.mark.parametrize("seed", range(8))
def test_oracle_vs_pyref_random_corruption(seed):
    rng = random.Random(seed)
    base = 1_700_000_000
    w = P.PyWal(base, base)
    for i in range(25):
        ns, key, val, etag, expire, tomb, meta = _rand_record(rng, base)
        w.write_record(P.record_encode(ns, key, val[:3000], etag, expire, tomb, meta, base))
    data = bytearray(w.buf)
    for _ in range(rng.randrange(0, 3)):
        data[rng.randrange(40, len(data))] ^= 1 << rng.randrange(8)
    if rng.random() < 0.3:
        data = data[:rng.randrange(40, len(data))]
    data = bytes(data)
    a = O.decode(data, 40, base, 20, 20)
    b = P.iterate(data, 40, base, 20, 20)
    assert a.err_class == b["err_class"]
    assert len(a.frags) == len(b["frags"])
    assert [int(x) for x in a.frags["crc_ok"]] == [f["crc_ok"] for f in b["frags"]]
    assert len(a.recs) == len(b["recs"])
    for got, want in zip(a.recs, b["recs"]):
        for k in ("foff", "size", "status", "first_frag", "emit_frag", "key_len", "expire"):
            assert int(got[k]) == (want[k] & 0xFFFFFFFFFFFFFFFF), k


def test_hint_codec_parity():
    rng = random.Random(7)
    for _ in range(50):
        ns = bytes(rng.getrandbits(8) for _ in range(20))
        key = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        fid, off, size = rng.randrange(1 << 20), rng.randrange(1 << 40), rng.randrange(1 << 20)
        a = O.hint_encode(ns, key, fid, off, size)
        assert a == P.hint_encode(ns, key, fid, off, size)
        st, f = P.hint_decode(a, 20)
        assert st == 0 and (f["fid"], f["off"], f["size"]) == (fid, off, size)


def test_synth_counts():
    data = O.synth(2 << 20, 0, 0x5EED)
    d = O.decode(data, 40, 1_700_000_000, 20, 20, want_bytes=False)
    assert d.err_class == 0 and (d.recs["status"] == 0).all()
    assert (d.recs["size"] == 4222).all()  # 26 B header + 100 B key + 4096 B value
    n, ec, _ = O.decode_fast(data, 40, 1_700_000_000, 20, 20)
    assert n == len(d.recs) and ec == 0


def _py_meta_zero(m: bytes) -> bool:
    """canonical msgpack empty maps (AppMetaSize 0): nil, {}, fixmap of empty strings / nils"""
    if len(m) == 1:
        return m[0] in (0xc0, 0x80)
    return len(m) >= 3 and (m[0] & 0xf0) == 0x80 and len(m) == 1 + 2 * (m[0] & 15) and all(b in (0xa0, 0xc0) for b in m[1:])


def _py_compact(data, keep, dst, hint, fid, src_base, dst_base, ns_size, etag_size):
    """compactOneWal (compaction.go:294-327) restated over pyref: (err_class, err_rec, offs)."""
    it = P.iterate(data, 40, src_base, ns_size, etag_size)
    offs = []
    for i, r in enumerate(it["recs"]):
        if r["status"] != 0:
            return 1, i, offs
        if not keep[i]:
            offs.append(None)
            continue
        p = r["payload"]
        ns = p[1:1 + ns_size]
        el = 0 if r["flags"] & 1 else etag_size
        etag = p[r["etag_off"]:r["etag_off"] + el]
        h, kl, vl, ml = r["hdr_size"], r["key_len"], r["val_len"], r["meta_len"]
        key, val, meta = p[h:h + kl], p[h + kl:h + kl + vl], p[h + kl + vl:h + kl + vl + ml]
        if _py_meta_zero(meta):
            meta = b""
        exp = r["expire"]
        if exp != 0 and exp < dst_base:
            return 2, i, offs
        if exp != 0 and exp - dst_base >= 1 << 35:
            return 3, i, offs
        enc = P.record_encode(ns, key, val, etag, exp, bool(r["flags"] & 4), meta, dst_base)
        o = dst.write_record(enc)
        offs.append(o)
        hint.write_record(P.hint_encode(ns, key, fid, o, len(enc)))
    return (1 if it["err_class"] else 0), -1, offs


@pytest.mark.parametrize("seed", range(6))
def test_compact_oracle_vs_pyref(seed):
    rng = random.Random(300 + seed)
    base = 1_700_000_000
    w = P.PyWal(base, base)
    recs = []
    for i in range(30):
        ns, key, val, etag, expire, tomb, meta = _rand_record(rng, base)
        if rng.random() < 0.1:
            meta = rng.choice([b"\x80", b"\xc0", b"\x81\xa0\xa0"])
        enc = P.record_encode(ns, key, val[:3000], etag, expire, tomb, meta, base)
        if enc is not None:
            recs.append(enc)
            w.write_record(enc)
    data = bytearray(w.buf)
    if seed % 3 == 2:
        data[rng.randrange(40, len(data))] ^= 4
    data = bytes(data)
    keep = [rng.random() < 0.7 for _ in recs]
    dst_base = base - rng.choice([0, 10, 1 << 36]) if seed % 2 else base + rng.choice([0, 3])
    pd, ph = P.PyWal(1, dst_base), P.PyWal(1, dst_base)
    ec, er, offs = _py_compact(data, keep, pd, ph, 9, base, dst_base, 20, 20)
    od, oh = O.Writer(1, dst_base), O.Writer(1, dst_base)
    oec, oer, nin, ooffs = O.compact_append(od, oh, 9, data, 40, base, dst_base, 20, 20,
                                            np.array(keep, dtype=np.uint8))
    assert (oec, oer) == (ec, er)
    assert od.data() == bytes(pd.buf) and oh.data() == bytes(ph.buf)
    for i, o in enumerate(offs):
        assert (o is None and ooffs[i] == np.iinfo(np.uint64).max) or o == ooffs[i]


def test_meta_app_size_zero_and_expire_panic():
    for m, z in [(b"\x80", 1), (b"\xc0", 1), (b"\x81\xa0\xa0", 1), (b"\x82\xa0\xc0\xc0\xa0", 1), (b"\x81\xa1k\xa0", 0),
                 (b"", 0), (b"\x81\xa0", 0), (b"\x90", 0)]:
        assert O.meta_app_size_zero(m) == bool(z) == _py_meta_zero(m) or (m == b"" and not O.meta_app_size_zero(m))
    base = 1_700_000_000
    assert O.record_encode(b"", b"k", b"v", b"", base + (1 << 35) - 1, False, b"", base) is not None
    assert O.record_encode(b"", b"k", b"v", b"", base + (1 << 35), False, b"", base) is None  # reference panics


def test_writer_virtual_start():
    """oc_writer_new_at (the large-offset encode tests' reference): a writer opened at file size P keeps none of the
    first P bytes but lays out and returns offsets exactly as a writer that really wrote them (wal.go:482-516)"""
    BASE = 1_700_000_000
    rng = random.Random(11)
    for target in (40, 41, 32768 + 40 - 7, 3 * 32768 + 123, 5 * 32768 + 40 - 3):
        w = O.Writer(BASE, BASE)
        while w.size() < target:
            w.write(bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, min(5000, target - w.size() + 8)))))
        P = w.size()
        v = O.Writer(BASE, BASE, at=P)
        assert v.size() == P and v.base() == P
        for _ in range(40):
            rec = bytes(rng.getrandbits(8) for _ in range(rng.choice([1, 6, 7, 100, 4222, 32761, 40000])))
            assert w.write(rec) == v.write(rec)
        assert w.size() == v.size() and w.data()[P:] == v.data()
