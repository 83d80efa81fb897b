"""WAL test inputs mirroring the reference tests plus the branch fixtures SURVEY.md 4 asks for.
Built with the oracle writer (tests only). Each builder returns (file_bytes, params dict)."""
from __future__ import annotations

import hashlib
import random

import numpy as np

import _oracle as O

BASE = 1_700_000_000


def sha1(s: str) -> bytes:
    return hashlib.sha1(s.encode()).digest()


def params(ns=20, etag=20, start_off=40, base=BASE, mode=0):
    return dict(ns_size=ns, etag_size=etag, start_off=start_off, base_time=base, mode=mode)


def wal_of(payloads, base=BASE, create=None):
    w = O.Writer(create if create is not None else base, base)
    offs = [w.write(p) for p in payloads]
    return w.data(), offs


def rec(i, vlen=11, ns=20, etag=b"", expire=0, tomb=False, meta=b"", base=BASE, klen=None):
    key = (b"key-%06d" % i) if klen is None else bytes((i * 7 + k) & 0xff for k in range(klen))
    rng = random.Random(i)
    val = bytes(rng.getrandbits(8) for _ in range(vlen))
    return O.record_encode(sha1("ns")[:ns] if ns <= 20 else bytes(ns), key, val, etag, expire, tomb, meta, base)


# --- reference test scenarios (restated) ---
def case_iterator_basic():
    """wal_iterator_test.go:11-40: 1000 tiny payloads "0".."999" (not valid records: invalid data)."""
    data, _ = wal_of([str(i).encode() for i in range(1000)])
    return data, params()


def case_iterator_large():
    """wal_iterator_test.go:42-74: 1024 x 5 KiB payloads (spanning records)."""
    blob = (b"01234567" * 128) * 5
    data, _ = wal_of([blob] * 1024)
    return data, params()


def case_large_record():
    """wal_test.go:73-94: one 64 KiB record -> First/Middle/Last."""
    data, _ = wal_of([bytes(i % 256 for i in range(65536))])
    return data, params()


def case_records_mixed():
    """record_test.go:43-147 shapes (etag, expire, tombstone, meta, empty value) inside a WAL."""
    etag = sha1("etag")
    ps = []
    for i in range(300):
        k = i % 4
        if k == 0:
            ps.append(rec(i, 11, etag=etag, expire=BASE + 60, tomb=True, meta=b"\x81\xa3foo\xa3bar"))
        elif k == 1:
            ps.append(rec(i, 11, etag=etag, expire=BASE + 61))
        elif k == 2:
            ps.append(rec(i, 0, etag=etag, expire=BASE + 62, tomb=True, meta=b"\x81\xa3foo\xa3bar"))
        else:
            ps.append(rec(i, 0))
    data, _ = wal_of(ps)
    return data, params()


def case_config_shape(n=400, vlen=4096):
    """config A/B shape: ns 20, key 100, value 4096, no etag/expire/meta."""
    data, _ = wal_of([rec(i, vlen, klen=100) for i in range(n)])
    return data, params()


# --- branch fixtures ---
def case_padding():
    """leftover < 7 at a block end (wal.go:507-512): first record leaves 3 bytes in block 0."""
    first = bytes(32768 - 7 - 3)  # 32758 B record -> 32765 bytes used, 3 left -> padding
    data, _ = wal_of([first, rec(1, 100), rec(2, 50000), rec(3, 10)])
    return data, params()


def case_zero_first():
    """leftover == 7 (wal.go:518-519): a zero-length First fragment, offset re-captured."""
    first = bytes(32768 - 7 - 7)  # leaves exactly 7 bytes
    data, _ = wal_of([first, rec(1, 200), rec(2, 10)])
    return data, params()


def case_zipf(n=600, seed=42):
    rng = np.random.default_rng(seed)
    ps = [rec(i, int(128 * min(rng.zipf(1.1), 512)), klen=100) for i in range(n)]
    data, _ = wal_of(ps)
    return data, params()


def case_sparse_multi(n=6000, seed=7):
    """Long runs of single-window fragments between rare multi-window ones: a 64-fragment window
    can hold few body windows, so one CRC pass spans many fragment windows."""
    rng = np.random.default_rng(seed)
    ps = []
    for i in range(n):
        r = rng.random()
        v = int(rng.integers(200, 70000)) if r < 0.03 else int(rng.integers(1, 60))
        ps.append(rec(i, v, klen=int(rng.integers(1, 40))))
    data, _ = wal_of(ps)
    return data, params()


def case_tail_garbage():
    """file with < 7 trailing bytes after the last fragment (ignored) and a truncated last block."""
    data, _ = wal_of([rec(i, 300) for i in range(20)])
    return data + b"\x01\x02\x03", params()


def case_truncated_record():
    """a First fragment at EOF without its Last: silently dropped (ErrWalIteratorEOF)."""
    data, _ = wal_of([rec(0, 100), rec(1, 40000)])
    return data[:40 + 32768 + 100], params()


def case_zero_tail():
    """an all-zero region after valid data: masked CRC of empty != 0 -> CRC error."""
    data, _ = wal_of([rec(i, 100) for i in range(5)])
    return data + bytes(64), params()


def case_bad_type():
    """valid CRC, unknown type byte 9 (ErrWalUnknownRecordType)."""
    data, _ = wal_of([rec(i, 100) for i in range(5)])
    b = bytearray(data)
    # rewrite the 3rd fragment's type: header offsets follow Full records of equal size
    flen = len(rec(0, 100))
    h = 40 + 2 * (7 + flen)
    b[h + 6] = 9
    return bytes(b), params()


def case_out_of_order():
    """Middle/Last without First, Full after First, First after First (crafted, valid CRCs)."""
    w = O.Writer(BASE, BASE)
    # hand-frame fragments: use the writer on pieces then patch types
    pieces = [rec(0, 50), rec(1, 60), rec(2, 70), rec(3, 80), rec(4, 90), rec(5, 30)]
    offs = [w.write(p) for p in pieces]
    b = bytearray(w.data())
    b[offs[0] + 6] = 4   # Last with no First: emitted alone
    b[offs[1] + 6] = 2   # First ...
    b[offs[2] + 6] = 1   # ... then Full: Full's data with First's offset
    b[offs[3] + 6] = 2   # First
    b[offs[4] + 6] = 2   # First again (appended)
    b[offs[5] + 6] = 4   # Last: concatenation of 3 fragments -> invalid data
    return bytes(b), params()


def case_clamped():
    """a length field larger than the block: clamped (wal_iterator.go:75), then CRC fails."""
    data, _ = wal_of([rec(i, 100) for i in range(3)])
    b = bytearray(data)
    b[40 + 4] = 0xff
    b[40 + 5] = 0xff
    return bytes(b), params()


def case_start_off(delta):
    data, _ = wal_of([rec(i, 500) for i in range(100)])
    return data, params(start_off=40 + delta)


def case_panic_records():
    """records that make RecordFromBytes panic or fail validation."""
    ns = 20
    good = rec(0, 10)
    # expire flag clear but etag field extends beyond the data
    p1 = bytearray(good)
    p1[1 + ns] = 0  # flags: etag present, expire present
    # keyLen huge so that the uint64 sum wraps
    hdr = bytes([0]) + sha1("ns")[:ns] + bytes([3])
    big = O.put_uvarint(1 << 63) + O.put_uvarint(1 << 63) + O.put_uvarint(0)
    body = hdr + big
    p2 = bytearray(body)
    p2[0] = len(body) & 0xff
    # length exactly min header (1+ns+1+3) with mismatching header size
    p3 = bytes([9]) + bytes(ns) + bytes([3, 0, 0, 0])
    data, _ = wal_of([good, bytes(p1), bytes(p2), p3, bytes(4), rec(5, 10)])
    return data, params()


def case_hint(n=500):
    """a hint WAL rebuilt from a data WAL (hint.go:123-161)."""
    data, p = case_config_shape(n, 300)
    ec, _, _, hint = O.hint_by_wal(data, 7, 40, BASE, 20, 20)
    assert ec == 0
    return hint, params(mode=1)


def corrupt(data: bytes, rng: random.Random, nflips: int = 1) -> bytes:
    b = bytearray(data)
    for _ in range(nflips):
        i = rng.randrange(40, len(b))
        b[i] ^= 1 << rng.randrange(8)
    return bytes(b)


ALL = {
    "iterator_basic": case_iterator_basic,
    "iterator_large": case_iterator_large,
    "large_record": case_large_record,
    "records_mixed": case_records_mixed,
    "config_shape": case_config_shape,
    "padding": case_padding,
    "zero_first": case_zero_first,
    "zipf": case_zipf,
    "sparse_multi": case_sparse_multi,
    "sparse_multi_dense": lambda: case_sparse_multi(4000, 11),
    "tail_garbage": case_tail_garbage,
    "truncated_record": case_truncated_record,
    "zero_tail": case_zero_tail,
    "bad_type": case_bad_type,
    "out_of_order": case_out_of_order,
    "clamped": case_clamped,
    "start_off_plus4": lambda: case_start_off(4),
    "start_off_plus7": lambda: case_start_off(7),
    "start_off_minus40": lambda: case_start_off(-40),
    "start_off_beyond": lambda: case_start_off(10_000_000),
    "panic_records": case_panic_records,
    "hint": case_hint,
}
