"""Generates the committed golden fixtures with the independent Python restatement (pyref.py).

Each fixture is <name>.wal (the file image) + <name>.json (decode parameters and the expected
iterator output: fragments, records with parsed fields, payload SHA-1, first error). The C oracle
and the GPU codec are both tested against these files. Run: python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import struct

import pyref as P

HERE = os.path.dirname(os.path.abspath(__file__))
BASE = 1_700_000_000
NS = hashlib.sha1(b"test-ns").digest()
ETAG = hashlib.sha1(b"etag").digest()


def rec(i, vlen=11, etag=b"", expire=0, tomb=False, meta=b""):
    rng = random.Random(1000 + i)
    return P.record_encode(NS, b"test-key-%d" % i, bytes(rng.getrandbits(8) for _ in range(vlen)), etag, expire, tomb,
                           meta, BASE)


def wal(payloads, create=BASE, base=BASE):
    w = P.PyWal(create, base)
    for p in payloads:
        w.write_record(p)
    return bytes(w.buf)


def fixtures():
    out = {}
    # wal_iterator_test.go:11-40 and wal_test.go:17-70 scenarios
    out["basic_tiny"] = (wal([str(i).encode() for i in range(1000)]), {})
    out["multiple_records"] = (wal([b"first record", b"second record", b"third record"]), {})
    # record_test.go:43-147 shapes
    ps = []
    for i in range(40):
        k = i % 5
        if k == 0:
            ps.append(rec(i, 11, ETAG, BASE + 60, True, b"\x81\xa3foo\xa3bar"))
        elif k == 1:
            ps.append(rec(i, 11, ETAG, BASE + 61))
        elif k == 2:
            ps.append(rec(i, 0, ETAG, BASE + 62, True, b"\x81\xa3foo\xa3bar"))
        elif k == 3:
            ps.append(rec(i, 0))
        else:
            ps.append(rec(i, 3000, b"", BASE + 300000))  # 3-byte expire varint
    out["records_mixed"] = (wal(ps), {})
    # TestRecord_EmptyNs: ns 0, etag 0
    ps = [P.record_encode(b"", b"test-key", b"test-value", b"", 0, False, b"", BASE) for _ in range(5)]
    out["empty_ns"] = (wal(ps), {"ns_size": 0, "etag_size": 0})
    # wal_test.go:73-94 large record -> First / Middle / Last
    out["large_record"] = (wal([bytes(i % 256 for i in range(2 * 32768))]), {})
    # padding (leftover < 7) and zero-length First (leftover == 7): SURVEY.md 4 branch gaps
    out["padding"] = (wal([bytes(32768 - 7 - 3), rec(1, 100), rec(2, 40000), rec(3, 5)]), {})
    out["zero_first"] = (wal([bytes(32768 - 7 - 7), rec(1, 200), rec(2, 10)]), {})
    # TestWal_CorruptedRead: overwrite 2 bytes at offset+2 (inside the CRC field)
    w = P.PyWal(BASE, BASE)
    offs = [w.write_record(rec(i, 50)) for i in range(6)]
    b = bytearray(w.buf)
    b[offs[3] + 2:offs[3] + 4] = b"\xde\xad"
    out["corrupted_crc"] = (bytes(b), {})
    # unknown type with a valid CRC
    b = bytearray(w.buf)
    b[offs[2] + 6] = 7
    out["bad_type"] = (bytes(b), {})
    # out-of-order types with valid CRCs (crafted)
    w2 = P.PyWal(BASE, BASE)
    o2 = [w2.write_record(rec(i, 40 + i)) for i in range(6)]
    b = bytearray(w2.buf)
    for k, t in zip(range(6), (4, 2, 1, 2, 2, 4)):
        b[o2[k] + 6] = t
    out["out_of_order"] = (bytes(b), {})
    # length field larger than the block: clamp then CRC mismatch
    b = bytearray(wal([rec(i, 60) for i in range(3)]))
    b[44:46] = b"\xff\xff"
    out["clamped_length"] = (bytes(b), {})
    # all-zero tail, short tail, truncated file
    base = wal([rec(i, 80) for i in range(4)])
    out["zero_tail"] = (base + bytes(32), {})
    out["short_tail"] = (base + b"\x05\x06\x07", {})
    out["truncated"] = (wal([rec(0, 100), rec(1, 40000)])[:40 + 32768 + 50], {})
    # RecordFromBytes panics / invalid data
    good = rec(0, 10)
    p1 = bytearray(good)
    p1[1 + 20] = 0
    hdr = bytes([0]) + NS + bytes([3])
    body = bytearray(hdr + P.put_uvarint(1 << 63) + P.put_uvarint(1 << 63) + P.put_uvarint(0))
    body[0] = len(body)
    out["panic_records"] = (wal([good, bytes(p1), bytes(body), bytes([9]) + bytes(20) + bytes([3, 0, 0, 0]),
                                 bytes(4), rec(5, 10)]), {})
    # start offsets other than 40 (the loader does not validate startOff, wal.go:381)
    base = wal([rec(i, 300) for i in range(30)])
    out["start_off_44"] = (base, {"start_off": 44})
    out["start_off_beyond"] = (base, {"start_off": len(base) + 5})
    # hint file built like NewHintByWal (hint.go:123-161)
    data = wal([rec(i, 700) for i in range(60)])
    it = P.iterate(data, 40, BASE, 20, 20)
    hw = P.PyWal(BASE, BASE)
    for r in it["recs"]:
        pl = r["payload"]
        hw.write_record(P.hint_encode(pl[1:21], pl[r["hdr_size"]:r["hdr_size"] + r["key_len"]], 3, r["foff"] - 7,
                                      r["size"]))
    out["hint"] = (bytes(hw.buf), {"mode": 1})
    hb = bytearray(hw.buf)
    hb[40 + 7 + 20] = 0xF0  # corrupt a key length varint: CRC now fails
    out["hint_corrupt"] = (bytes(hb), {"mode": 1})
    return out


def expected(data, prm):
    p = dict(start_off=40, base_time=BASE, ns_size=20, etag_size=20, mode=0)
    p.update(prm)
    it = P.iterate(data, p["start_off"], p["base_time"], p["ns_size"], p["etag_size"], p["mode"])
    recs = []
    for r in it["recs"]:
        r = dict(r)
        r["payload_sha1"] = hashlib.sha1(r.pop("payload")).hexdigest()
        recs.append(r)
    return dict(params=p, frags=it["frags"], recs=recs, err_class=it["err_class"], err_frag=it["err_frag"],
                file_sha1=hashlib.sha1(data).hexdigest(), size=len(data))


def main():
    for name, (data, prm) in fixtures().items():
        assert len(data) < 256 * 1024, name
        with open(os.path.join(HERE, name + ".wal"), "wb") as f:
            f.write(data)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(expected(data, prm), f, indent=0, sort_keys=True)
        print(name, len(data))


if __name__ == "__main__":
    main()
