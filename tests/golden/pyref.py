"""Independent pure-Python restatement of the reference WAL codec (TEST INFRASTRUCTURE ONLY).

Written directly from the Go sources of wenzhang-dev/bitcaskDB, separately from oracle/bcw_oracle.c,
so the two restatements cross-check each other (the Go toolchain is absent from this image):
  utils.go:24-29 ComputeCRC32 (bitwise CRC-32C here, no tables), utils.go:51-57 DecodeUvarint,
  wal.go:332-360 writeSuperBlock, wal.go:490-553 WriteRecord, wal_iterator.go:40-100 Next,
  record.go:57-138 Encode, record.go:140-239 RecordFromBytes, hint.go:32-84 hint codec.
Small inputs only (pure Python loops)."""
from __future__ import annotations

import struct

MASK64 = (1 << 64) - 1


def crc32c_bitwise(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def compute_crc32(data: bytes) -> int:
    c = crc32c_bitwise(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def go_uvarint(buf: bytes):
    """encoding/binary.Uvarint (go1.24)."""
    x, s = 0, 0
    for i, b in enumerate(buf):
        if i == 10:
            return 0, -(i + 1)
        if b < 0x80:
            if i == 9 and b > 1:
                return 0, -(i + 1)
            return x | (b << s), i + 1
        x |= (b & 0x7F) << s
        s += 7
    return 0, 0


def decode_uvarint(buf: bytes):
    v, n = go_uvarint(buf)
    return (0, 0) if n <= 0 else (v, n)


def put_uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def super_block(create_time: int, base_time: int) -> bytes:
    b = struct.pack("<QQIQQ", 0x77616C64, 32768, 40, create_time, base_time)
    return b + struct.pack("<I", compute_crc32(b))


class PyWal:
    def __init__(self, create_time: int, base_time: int):
        self.buf = bytearray(super_block(create_time, base_time))

    def write_record(self, record: bytes) -> int:
        offset, begin, left = 0, True, len(record)
        while left > 0:
            leftover = 32768 - ((len(self.buf) - 40) % 32768)
            if leftover < 7:
                self.buf += bytes(leftover)
                leftover = 32768
            if begin:
                offset = len(self.buf)
            frag = min(left, leftover - 7)
            end = left == frag
            rtype = 1 if begin and end else 2 if begin else 4 if end else 3
            self.buf += struct.pack("<IHB", compute_crc32(record[:frag]), frag, rtype) + record[:frag]
            record = record[frag:]
            left -= frag
            begin = False
        return offset


def record_encode(ns, key, value, etag=b"", expire=0, tombstone=False, meta=b"", base_time=0):
    flag = (1 if not etag else 0) | (4 if tombstone else 0)
    exp = b""
    if expire == 0:
        flag |= 2
    elif expire < base_time:
        return None
    elif expire - base_time >= 1 << 35:  # PutUvarint into a [MaxVarintLen32]byte array panics
        return None
    else:
        exp = put_uvarint(expire - base_time)
    v = put_uvarint(len(key)) + put_uvarint(len(value)) + put_uvarint(len(meta))
    header = len(v) + len(exp) + len(ns) + len(etag) + 2
    return bytes([header & 0xFF]) + ns + bytes([flag]) + v + etag + exp + key + value + meta


def _i64(x):
    x &= MASK64
    return x - (1 << 64) if x >> 63 else x


def record_from_bytes(data: bytes, base_time: int, ns_size: int, etag_size: int):
    """returns (status, fields): status 0 ok, 1 invalid data, 2 panic, 3 unsupported"""
    f = dict(hdr_size=0, flags=0, etag_off=0, key_len=0, val_len=0, meta_len=0, expire=0)
    if len(data) < 1 + ns_size + 1 + 3:
        return 1, f
    header = data[0]
    off = 1 + ns_size
    flag = data[off]
    off += 1
    kl, n = decode_uvarint(data[off:]); off += n
    vl, n = decode_uvarint(data[off:]); off += n
    ml, n = decode_uvarint(data[off:]); off += n
    f.update(hdr_size=header, flags=flag, etag_off=off & 0xFF, key_len=kl, val_len=vl, meta_len=ml)
    etag_len = 0 if flag & 1 else etag_size
    exp_size, expire = 0, 0
    if not flag & 2:
        if off + etag_len > len(data):
            return 2, f
        expire, exp_size = decode_uvarint(data[off + etag_len:])
        expire = (expire + base_time) & MASK64
    f["expire"] = expire
    cur_hdr = off + etag_len + exp_size
    cur_total = _i64(cur_hdr + _i64(kl + vl + ml))
    if cur_hdr != header or cur_total != len(data):
        return 1, f
    if kl >> 63 or vl >> 63 or ml >> 63 or kl + vl + ml > MASK64:
        return 2, f
    if max(kl, vl, ml, len(data)) > 0xFFFFFFFF:
        return 3, f
    return 0, f


def hint_encode(ns, key, fid, off, size):
    return ns + put_uvarint(len(key)) + key + put_uvarint(fid) + put_uvarint(off) + put_uvarint(size)


def hint_decode(data: bytes, ns_size: int):
    f = dict(hdr_size=0, key_len=0, fid=0, off=0, size=0)
    if len(data) < ns_size + 5:
        return 1, f
    off = ns_size
    kl, n = decode_uvarint(data[off:]); off += n
    key_off = off
    off = _i64(off + kl)
    f.update(key_len=kl, hdr_size=key_off & 0xFF)
    if off < 0 or off > len(data):
        return 2, f
    fid, n = decode_uvarint(data[off:]); off += n
    ho, n = decode_uvarint(data[off:]); off += n
    hs, n = decode_uvarint(data[off:]); off += n
    f.update(fid=fid, off=ho, size=hs)
    if off != len(data):
        return 1, f
    if kl >> 63:
        return 2, f
    return 0, f


def iterate(data: bytes, start_off: int, base_time: int, ns_size: int, etag_size: int, mode: int = 0):
    """WalIterator.Next driven to EOF/first fragment error; every emitted record is parsed.
    Returns dict(frags=[...], recs=[...], err_class, err_frag)."""
    frags, recs = [], []
    size = len(data)
    file_off, buf_off, buf_size = start_off, 0, 0
    record = bytearray()
    off = first = 0
    while True:
        if buf_off + 7 > buf_size:
            file_off += buf_size
            buf_size = min(32768, size - file_off)
            if buf_size == 0:
                return dict(frags=frags, recs=recs, err_class=0, err_frag=None)
            if buf_size < 0:
                return dict(frags=frags, recs=recs, err_class=3, err_frag=None)
            buf_off = 0
            if buf_size < 7:  # header sliced from the stale 32 KiB buffer, then buf[7:7+neg] panics
                return dict(frags=frags, recs=recs, err_class=3, err_frag=None)
        buf = data[file_off:file_off + buf_size]
        crc, length, rtype = struct.unpack_from("<IHB", buf, buf_off)
        buf_off += 7
        if len(record) == 0:
            off, first = file_off + buf_off, len(frags)
        length = min(length, buf_size - buf_off)
        frag = buf[buf_off:buf_off + length]
        ok = compute_crc32(frag) == crc
        frags.append(dict(data_off=file_off + buf_off, len=length, stored_crc=crc, type=rtype, crc_ok=int(ok)))
        buf_off += length
        gi = len(frags) - 1
        if not ok:
            return dict(frags=frags, recs=recs, err_class=1, err_frag=gi)
        if rtype == 1:
            payload, f0 = bytes(frag), gi
        elif rtype in (2, 3, 4):
            record += frag
            if rtype != 4:
                continue
            payload, f0 = bytes(record), first
        else:
            return dict(frags=frags, recs=recs, err_class=2, err_frag=gi)
        if mode == 0:
            st, fields = record_from_bytes(payload, base_time, ns_size, etag_size)
        else:
            st, fields = hint_decode(payload, ns_size)
        recs.append(dict(foff=off, size=len(payload), first_frag=f0, emit_frag=gi, status=st, payload=payload,
                         **{("hint_size" if k == "size" else k): v for k, v in fields.items()}))
        record = bytearray()


# ---- index hash: spaolacci/murmur3 v1.1.0 New64().Sum64() (index.go:15-19), independent restatement ----
_M64 = (1 << 64) - 1


def _rotl64(x, r):
    return ((x << r) | (x >> (64 - r))) & _M64


def _fmix64(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & _M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & _M64
    k ^= k >> 33
    return k


def murmur3_x64_128(data: bytes, seed: int = 0):
    c1, c2 = 0x87c37b91114253d5, 0x4cf5ad432745937f
    h1 = h2 = seed & _M64
    n = len(data)
    nb = n // 16
    for i in range(nb):
        k1 = int.from_bytes(data[16 * i:16 * i + 8], "little")
        k2 = int.from_bytes(data[16 * i + 8:16 * i + 16], "little")
        k1 = (_rotl64((k1 * c1) & _M64, 31) * c2) & _M64
        h1 ^= k1
        h1 = (_rotl64(h1, 27) + h2) & _M64
        h1 = (h1 * 5 + 0x52dce729) & _M64
        k2 = (_rotl64((k2 * c2) & _M64, 33) * c1) & _M64
        h2 ^= k2
        h2 = (_rotl64(h2, 31) + h1) & _M64
        h2 = (h2 * 5 + 0x38495ab5) & _M64
    tail = data[16 * nb:]
    if len(tail) > 8:
        k2 = int.from_bytes(tail[8:], "little")
        h2 ^= (_rotl64((k2 * c2) & _M64, 33) * c1) & _M64
    if len(tail) > 0:
        k1 = int.from_bytes(tail[:8], "little")
        h1 ^= (_rotl64((k1 * c1) & _M64, 31) * c2) & _M64
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & _M64
    h2 = (h2 + h1) & _M64
    h1, h2 = _fmix64(h1), _fmix64(h2)
    h1 = (h1 + h2) & _M64
    h2 = (h2 + h1) & _M64
    return h1, h2


def murmur3_sum64(data: bytes) -> int:
    return murmur3_x64_128(data)[0]


class PyIndex:
    """Index semantics (index.go:81-165): MergedKey(ns, key) -> (fid, off, size); Get reports
    not-found / soft-deleted (off == 0). No eviction (capacity >= keys)."""

    def __init__(self):
        self.m = {}

    def put(self, ns, key, fid, off, size):
        self.m[bytes(ns) + bytes(key)] = (fid, off, size)

    def delete(self, ns, key):
        self.m.pop(bytes(ns) + bytes(key), None)

    def soft_delete(self, ns, key):
        self.m[bytes(ns) + bytes(key)] = (0, 0, 0)

    def get(self, ns, key):
        v = self.m.get(bytes(ns) + bytes(key))
        if v is None:
            return 1, None
        return (2 if v[1] == 0 else 0), v

    def do_filter(self, ns, key, src_fid, src_off) -> bool:
        """compaction.go:329-348 (no user filter): True drops the record."""
        st, v = self.get(ns, key)
        return st != 0 or v[0] != src_fid or v[1] != src_off
