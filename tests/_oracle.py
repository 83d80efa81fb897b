"""ctypes binding of the CPU parity oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# ORACLE_LIB: an alternative build of the same oracle (the ASan/UBSan one of tools/sanitize_cpu.sh)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")

FRAG_DT = np.dtype([("data_off", "<u8"), ("len", "<u4"), ("stored_crc", "<u4"), ("type", "u1"), ("crc_ok", "u1"),
                    ("pad", "u1", 6)])
REC_DT = np.dtype([("foff", "<u8"), ("size", "<u8"), ("expire", "<u8"), ("key_len", "<u8"), ("val_len", "<u8"),
                   ("meta_len", "<u8"), ("first_frag", "<u4"), ("emit_frag", "<u4"), ("hdr_size", "u1"),
                   ("flags", "u1"), ("etag_off", "u1"), ("status", "u1"), ("pad", "u1", 4)])
assert FRAG_DT.itemsize == 24 and REC_DT.itemsize == 64


def _build():
    src = os.path.join(ORACLE_DIR, "bcw_oracle.c")
    if os.environ.get("ORACLE_LIB"):
        return
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)


_build()
lib = C.CDLL(LIB)
vp = C.c_void_p
lib.oc_compute_crc32.restype = C.c_uint32
lib.oc_compute_crc32.argtypes = [vp, C.c_size_t]
lib.oc_crc32c.restype = C.c_uint32
lib.oc_crc32c.argtypes = [vp, C.c_size_t]
lib.oc_crc32c_hw.restype = C.c_uint32
lib.oc_crc32c_hw.argtypes = [vp, C.c_size_t]
lib.oc_uvarint.restype = C.c_int
lib.oc_uvarint.argtypes = [vp, C.c_size_t, C.POINTER(C.c_uint64)]
lib.oc_put_uvarint.restype = C.c_int
lib.oc_put_uvarint.argtypes = [vp, C.c_uint64]
lib.oc_super_encode.argtypes = [vp, C.c_uint64, C.c_uint64]
lib.oc_writer_new.restype = vp
lib.oc_writer_new.argtypes = [C.c_uint64, C.c_uint64]
lib.oc_writer_write.restype = C.c_uint64
lib.oc_writer_write.argtypes = [vp, vp, C.c_size_t]
lib.oc_writer_size.restype = C.c_uint64
lib.oc_writer_size.argtypes = [vp]
lib.oc_writer_new_at.restype = vp
lib.oc_writer_new_at.argtypes = [C.c_uint64]
lib.oc_writer_base.restype = C.c_uint64
lib.oc_writer_base.argtypes = [vp]
lib.oc_writer_data.restype = vp
lib.oc_writer_data.argtypes = [vp]
lib.oc_writer_free.argtypes = [vp]
lib.oc_record_encode.restype = C.c_int64
lib.oc_record_encode.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, C.c_uint64,
                                 C.c_int, vp, C.c_size_t, C.c_uint64]
lib.oc_hint_encode.restype = C.c_size_t
lib.oc_hint_encode.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64]
lib.oc_decode_segment.restype = vp
lib.oc_decode_segment.argtypes = [vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int]
lib.oc_decode_counts.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
lib.oc_decode_frags.argtypes = [vp, vp]
lib.oc_decode_recs.argtypes = [vp, vp]
lib.oc_decode_bytes.argtypes = [vp, vp, vp]
lib.oc_decode_free.argtypes = [vp]
lib.oc_decode_fast.restype = C.c_uint64
lib.oc_decode_fast.argtypes = [vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                               C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
_i32p, _i64p, _u64p = C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_uint64)
lib.oc_compact_append.restype = None
lib.oc_compact_append.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32,
                                  C.c_uint32, vp, C.c_uint64, vp, _i32p, _i64p, _u64p]
lib.oc_hint_by_wal.restype = None
lib.oc_hint_by_wal.argtypes = [vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                               _i32p, _i64p, _u64p]
lib.oc_meta_app_size_zero.restype = C.c_int
lib.oc_meta_app_size_zero.argtypes = [vp, C.c_size_t]
lib.oc_wal_record_size.restype = C.c_uint64
lib.oc_wal_record_size.argtypes = [C.c_uint64, C.c_uint64]
lib.oc_wal_block_index_range.restype = None
lib.oc_wal_block_index_range.argtypes = [C.c_uint64, C.c_uint64, _u64p, _u64p, _u64p]
lib.oc_decode_payload_hashes.restype = None
lib.oc_decode_payload_hashes.argtypes = [vp, vp]
lib.oc_gather_payload_hashes.restype = None
lib.oc_gather_payload_hashes.argtypes = [vp, C.c_uint64, vp, vp, C.c_uint64, vp, vp, vp, C.c_uint64, vp]
lib.oc_murmur3_sum64.restype = C.c_uint64
lib.oc_murmur3_sum64.argtypes = [vp, C.c_size_t]
lib.oc_murmur3_128.restype = None
lib.oc_murmur3_128.argtypes = [vp, C.c_size_t, C.c_uint64, _u64p, _u64p]
lib.oc_index_new.restype = vp
lib.oc_index_new.argtypes = []
lib.oc_index_free.argtypes = [vp]
lib.oc_index_set.restype = None
lib.oc_index_set.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64]
lib.oc_index_get.restype = C.c_int
lib.oc_index_get.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, _u64p, _u64p, _u64p]
lib.oc_index_live.restype = C.c_uint64
lib.oc_index_live.argtypes = [vp]
lib.oc_do_filter.restype = C.c_int
lib.oc_do_filter.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, C.c_uint64, C.c_uint64]
lib.oc_index_put_segment.restype = C.c_int
lib.oc_index_put_segment.argtypes = [vp, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                     C.c_uint64, C.c_int, _u64p]
lib.oc_compact_filter.restype = C.c_uint64
lib.oc_compact_filter.argtypes = [vp, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, vp,
                                  C.c_uint64]
lib.oc_decode_fast_pread.restype = C.c_uint64
lib.oc_decode_fast_pread.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                     C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
lib.oc_read_record.restype = C.c_int
lib.oc_read_record.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, vp]
lib.oc_record_parse.restype = None
lib.oc_record_parse.argtypes = [vp, C.c_size_t, C.c_size_t, C.c_uint64, C.c_uint32, C.c_uint32, vp]
lib.oc_synth_segment.restype = vp
lib.oc_synth_segment.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                 C.c_uint64]

lib.oc_smap_new.restype = vp
lib.oc_smap_new.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, vp, C.c_uint64,
                            C.c_uint64]
lib.oc_smap_free.argtypes = [vp]
lib.oc_smap_set_now.argtypes = [vp, C.c_uint64]
lib.oc_smap_size.restype = C.c_uint64
lib.oc_smap_size.argtypes = [vp]
lib.oc_smap_set.restype = C.c_int
lib.oc_smap_set.argtypes = [vp, vp, C.c_size_t, vp, vp]
lib.oc_smap_get.restype = C.c_int
lib.oc_smap_get.argtypes = [vp, vp, C.c_size_t, vp]
lib.oc_smap_delete.restype = C.c_int
lib.oc_smap_delete.argtypes = [vp, vp, C.c_size_t, vp]
lib.oc_smap_export.restype = C.c_uint64
lib.oc_smap_export.argtypes = [vp, vp, C.c_uint64, vp, vp, C.c_uint64, _u64p]
lib.oc_bindex_op.restype = None
lib.oc_bindex_op.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, _u64p,
                             _u64p]
lib.oc_bindex_get.restype = C.c_int
lib.oc_bindex_get.argtypes = [vp, vp, C.c_size_t, vp, C.c_size_t, _u64p, _u64p, _u64p]
lib.oc_bindex_put_segment.restype = C.c_int
lib.oc_bindex_put_segment.argtypes = [vp, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_uint64, C.c_int, _u64p]
lib.oc_bindex_compact_filter.restype = C.c_uint64
lib.oc_bindex_compact_filter.argtypes = [vp, vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                         C.c_uint64, vp, C.c_uint64]


def _bytes_at(ptr, n: int) -> bytes:
    """n bytes at ptr (ctypes.string_at takes a C int size: images of 2 GiB and more need the buffer protocol)"""
    return bytes((C.c_uint8 * n).from_address(ptr)) if n else b""


def _ptr(a):
    if isinstance(a, (bytes, bytearray)):
        a = np.frombuffer(a, dtype=np.uint8)
    return a.ctypes.data_as(vp) if a.size else None


def compute_crc32(b: bytes) -> int:
    return int(lib.oc_compute_crc32(_ptr(b), len(b)))


def crc32c(b: bytes) -> int:
    return int(lib.oc_crc32c(_ptr(b), len(b)))


def crc32c_hw(b: bytes) -> int:
    return int(lib.oc_crc32c_hw(_ptr(b), len(b)))


def uvarint(b: bytes):
    v = C.c_uint64()
    n = lib.oc_uvarint(_ptr(b), len(b), C.byref(v))
    return int(v.value), int(n)


def put_uvarint(v: int) -> bytes:
    buf = (C.c_uint8 * 10)()
    n = lib.oc_put_uvarint(buf, v)
    return bytes(buf[:n])


class Writer:
    """oc_writer: WAL file image (wal.go:490-553)."""

    def __init__(self, create_time: int, base_time: int, at: int | None = None):
        """at: open the writer at file size `at` (>= 40) with none of those bytes kept (oc_writer_new_at): the
        appended bytes are data(), at file offsets [base(), size())"""
        self.h = lib.oc_writer_new(create_time, base_time) if at is None else lib.oc_writer_new_at(at)

    def write(self, rec: bytes) -> int:
        return int(lib.oc_writer_write(self.h, _ptr(rec), len(rec)))

    def size(self) -> int:
        return int(lib.oc_writer_size(self.h))

    def base(self) -> int:
        return int(lib.oc_writer_base(self.h))

    def data(self) -> bytes:
        return _bytes_at(lib.oc_writer_data(self.h), self.size() - self.base())

    def __del__(self):
        if getattr(self, "h", None):
            lib.oc_writer_free(self.h)
            self.h = None


def record_encode(ns: bytes, key: bytes, val: bytes, etag: bytes = b"", expire: int = 0, tombstone: bool = False,
                  meta: bytes = b"", base_time: int = 0):
    out = np.zeros(len(ns) + len(key) + len(val) + len(etag) + len(meta) + 64, dtype=np.uint8)
    n = lib.oc_record_encode(_ptr(out), _ptr(ns), len(ns), _ptr(key), len(key), _ptr(val), len(val), _ptr(etag),
                             len(etag), expire, int(tombstone), _ptr(meta), len(meta), base_time)
    return None if n < 0 else bytes(out[:n])


def hint_encode(ns: bytes, key: bytes, fid: int, off: int, size: int) -> bytes:
    out = np.zeros(len(ns) + len(key) + 64, dtype=np.uint8)
    n = lib.oc_hint_encode(_ptr(out), _ptr(ns), len(ns), _ptr(key), len(key), fid, off, size)
    return bytes(out[:n])


class Decoded:
    def __init__(self, frags, recs, err_frag, err_class, payloads, hashes=None):
        self.frags, self.recs, self.err_frag, self.err_class, self.payloads = frags, recs, err_frag, err_class, payloads
        self.hashes = hashes


def decode(seg, start_off: int, base_time: int, ns_size: int, etag_size: int, mode: int = 0,
           want_bytes: bool = True, want_hashes: bool = False) -> Decoded:
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    h = lib.oc_decode_segment(_ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, mode)
    nf, nr, ef, nb = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    ec = C.c_int32()
    lib.oc_decode_counts(h, C.byref(nf), C.byref(nr), C.byref(ef), C.byref(ec), C.byref(nb))
    frags = np.zeros(nf.value, dtype=FRAG_DT)
    recs = np.zeros(nr.value, dtype=REC_DT)
    if nf.value:
        lib.oc_decode_frags(h, frags.ctypes.data_as(vp))
    if nr.value:
        lib.oc_decode_recs(h, recs.ctypes.data_as(vp))
    payloads = None
    if want_bytes:
        buf = np.zeros(max(nb.value, 1), dtype=np.uint8)
        offs = np.zeros(nr.value + 1, dtype=np.uint64)
        lib.oc_decode_bytes(h, buf.ctypes.data_as(vp), offs.ctypes.data_as(vp))
        payloads = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(nr.value)]
    hashes = None
    if want_hashes:
        hashes = np.zeros(max(nr.value, 1), dtype=np.uint64)
        lib.oc_decode_payload_hashes(h, hashes.ctypes.data_as(vp))
        hashes = hashes[:nr.value]
    lib.oc_decode_free(h)
    return Decoded(frags, recs, int(ef.value), int(ec.value), payloads, hashes)


def gather_payload_hashes(seg, frags: dict, table: dict) -> np.ndarray:
    """Hash of every record payload gathered from a (device) fragment + record table, comparable with
    decode(..., want_hashes=True).hashes."""
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    d_off = np.ascontiguousarray(frags["data_off"], dtype=np.uint64)
    f_len = np.ascontiguousarray(frags["len"], dtype=np.uint32)
    first = np.ascontiguousarray(table["first_frag"], dtype=np.uint32)
    emit = np.ascontiguousarray(table["emit_frag"], dtype=np.uint32)
    size = np.ascontiguousarray(table["size"], dtype=np.uint64)
    n = int(first.size)
    out = np.zeros(max(n, 1), dtype=np.uint64)
    lib.oc_gather_payload_hashes(_ptr(seg), seg.size, _ptr(d_off), _ptr(f_len), d_off.size, _ptr(first), _ptr(emit),
                                 _ptr(size), n, out.ctypes.data_as(vp))
    return out[:n]


def wal_record_size(offset: int, size: int) -> int:
    return int(lib.oc_wal_record_size(offset, size))


def wal_block_index_range(offset: int, size: int):
    a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
    lib.oc_wal_block_index_range(offset, size, C.byref(a), C.byref(b), C.byref(c))
    return int(a.value), int(b.value), int(c.value)


def read_record(seg, offset: int, size: int, verify: bool = True):
    """Wal.ReadRecord (wal.go:556-573) -> (OC_RD_* status, payload bytes when OK)."""
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    out = np.zeros(max(size, 1), dtype=np.uint8)
    st = int(lib.oc_read_record(_ptr(seg), seg.size, offset, size, int(verify), out.ctypes.data_as(vp)))
    return st, (bytes(out[:size]) if st == 0 else None)


def record_parse(payload: bytes, base_time: int, ns_size: int, etag_size: int):
    """RecordFromBytes (record.go:140-239) -> one REC_DT row."""
    r = np.zeros(1, dtype=REC_DT)
    lib.oc_record_parse(_ptr(payload), len(payload), len(payload), base_time, ns_size, etag_size,
                        r.ctypes.data_as(vp))
    return r[0]


def decode_fast(seg, start_off, base_time, ns_size, etag_size):
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    ec = C.c_int32()
    cs = C.c_uint64()
    n = lib.oc_decode_fast(_ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, C.byref(ec), C.byref(cs))
    return int(n), int(ec.value), int(cs.value)


def decode_fast_pread(fd: int, length: int, start_off, base_time, ns_size, etag_size):
    ec = C.c_int32()
    cs = C.c_uint64()
    n = lib.oc_decode_fast_pread(fd, length, start_off, base_time, ns_size, etag_size, C.byref(ec), C.byref(cs))
    return int(n), int(ec.value), int(cs.value)


def synth(target_bytes: int, max_records: int, seed: int, ns_size: int = 20, key_len: int = 100,
          value_len: int = 4096, value_mode: int = 0, base_time: int = 1_700_000_000) -> bytes:
    h = lib.oc_synth_segment(target_bytes, max_records, seed, ns_size, key_len, value_len, value_mode, base_time)
    out = _bytes_at(lib.oc_writer_data(h), int(lib.oc_writer_size(h)))
    lib.oc_writer_free(h)
    return out


def hint_by_wal(seg, fid, start_off, base_time, ns_size, etag_size, create_time=None, writer=None):
    """NewHintByWal (hint.go:123-161). Returns (err_class, err_rec, n_in, hint file image)."""
    w = writer or Writer(create_time if create_time is not None else base_time, base_time)
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    ec, er, ni = C.c_int32(), C.c_int64(), C.c_uint64()
    lib.oc_hint_by_wal(w.h, fid, _ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, C.byref(ec),
                       C.byref(er), C.byref(ni))
    return int(ec.value), int(er.value), int(ni.value), w.data()


def compact_append(dst: "Writer", hint: "Writer", dst_fid: int, seg, start_off: int, src_base: int, dst_base: int,
                   ns_size: int, etag_size: int, keep):
    """compactOneWal (compaction.go:294-327) appending to the dst / hint writers.
    Returns (err_class, err_rec, n_in, offs) with offs[i] = dst offset of row i or 2**64-1."""
    seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
    keep = np.ascontiguousarray(keep, dtype=np.uint8)
    offs = np.full(max(keep.size, 1), np.iinfo(np.uint64).max, dtype=np.uint64)
    ec, er, ni = C.c_int32(), C.c_int64(), C.c_uint64()
    lib.oc_compact_append(dst.h, hint.h, dst_fid, _ptr(seg), seg.size, start_off, src_base, dst_base, ns_size,
                          etag_size, _ptr(keep), keep.size, offs.ctypes.data_as(vp), C.byref(ec), C.byref(er),
                          C.byref(ni))
    return int(ec.value), int(er.value), int(ni.value), offs[:keep.size]


def meta_app_size_zero(meta: bytes) -> bool:
    return bool(lib.oc_meta_app_size_zero(_ptr(meta), len(meta)))


def murmur3_sum64(b: bytes) -> int:
    return int(lib.oc_murmur3_sum64(_ptr(b), len(b)))


def murmur3_128(b: bytes, seed: int = 0):
    a, c = C.c_uint64(), C.c_uint64()
    lib.oc_murmur3_128(_ptr(b), len(b), seed, C.byref(a), C.byref(c))
    return int(a.value), int(c.value)


class Index:
    """oc_index: the reference index's Get/Put/Delete/SoftDelete semantics (index.go:81-165)."""
    PUT, DELETE, SOFT_DELETE = 0, 1, 2

    def __init__(self):
        self.h = lib.oc_index_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib.oc_index_free(self.h)
            self.h = None

    def set(self, ns: bytes, key: bytes, op: int, fid: int = 0, off: int = 0, size: int = 0):
        lib.oc_index_set(self.h, _ptr(ns), len(ns), _ptr(key), len(key), op, fid, off, size)

    def put(self, ns, key, fid, off, size):
        self.set(ns, key, 0, fid, off, size)

    def get(self, ns: bytes, key: bytes):
        f, o, s = C.c_uint64(), C.c_uint64(), C.c_uint64()
        st = lib.oc_index_get(self.h, _ptr(ns), len(ns), _ptr(key), len(key), C.byref(f), C.byref(o), C.byref(s))
        return int(st), (int(f.value), int(o.value), int(s.value))

    def live(self) -> int:
        return int(lib.oc_index_live(self.h))

    def put_segment(self, seg, start_off, base_time, ns_size, etag_size, mode, fid, use_rec_fid=False):
        seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
        n = C.c_uint64()
        ec = lib.oc_index_put_segment(self.h, _ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, mode, fid,
                                      int(use_rec_fid), C.byref(n))
        return int(ec), int(n.value)

    def compact_filter(self, seg, start_off, base_time, ns_size, etag_size, src_fid, n_rows):
        seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
        keep = np.zeros(max(n_rows, 1), dtype=np.uint8)
        nv = lib.oc_compact_filter(self.h, _ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, src_fid,
                                   keep.ctypes.data_as(vp), n_rows)
        return keep[:n_rows], int(nv)


class SMap:
    """oc_smap: map.go's SimpleMap (nshards=1) / ShardMap (nshards=16) with the sampled eviction, Rand and
    WallTime injected (scripted `rand_vals` cycled as v % n like map_test.go's mock, or a seeded stream)."""

    def __init__(self, capacity, limited, pool_cap, sample_keys, nshards=16, hash_mode=0, rand_vals=(), seed=1):
        rv = np.asarray(rand_vals, dtype=np.uint64)
        self.h = lib.oc_smap_new(nshards, capacity, limited, pool_cap, sample_keys, hash_mode,
                                 rv.ctypes.data_as(vp) if rv.size else None, rv.size, seed)
        if not self.h:
            raise ValueError("ErrMapOptions")

    def __del__(self):
        if getattr(self, "h", None):
            lib.oc_smap_free(self.h)
            self.h = None

    def set_now(self, seconds: int):
        lib.oc_smap_set_now(self.h, seconds)

    def size(self) -> int:
        return int(lib.oc_smap_size(self.h))

    def set(self, key: bytes, val):
        v = (C.c_uint64 * 3)(*(list(val) + [0, 0, 0])[:3])
        old = (C.c_uint64 * 3)()
        r = lib.oc_smap_set(self.h, _ptr(key), len(key), v, old)
        return int(r), tuple(int(x) for x in old)

    def get(self, key: bytes):
        v = (C.c_uint64 * 3)()
        r = lib.oc_smap_get(self.h, _ptr(key), len(key), v)
        return (None if r else tuple(int(x) for x in v))

    def delete(self, key: bytes):
        old = (C.c_uint64 * 3)()
        r = lib.oc_smap_delete(self.h, _ptr(key), len(key), old)
        return (None if r else tuple(int(x) for x in old))

    def export(self):
        kb = C.c_uint64()
        n = int(lib.oc_smap_export(self.h, None, 0, None, None, 0, C.byref(kb)))
        keys = np.zeros(max(int(kb.value), 1), dtype=np.uint8)
        koff = np.zeros(n + 1, dtype=np.uint64)
        vals = np.zeros(3 * max(n, 1), dtype=np.uint64)
        lib.oc_smap_export(self.h, keys.ctypes.data_as(vp), keys.size, koff.ctypes.data_as(vp),
                           vals.ctypes.data_as(vp), n, C.byref(kb))
        kbytes = keys.tobytes()
        return {kbytes[int(koff[i]):int(koff[i + 1])]: tuple(int(x) for x in vals[3 * i:3 * i + 3]) for i in range(n)}

    # Index over the bounded map (index.go:81-165)
    def index_op(self, ns: bytes, key: bytes, op: int, fid=0, off=0, size=0):
        ff, fb = C.c_uint64(), C.c_uint64()
        lib.oc_bindex_op(self.h, _ptr(ns), len(ns), _ptr(key), len(key), op, fid, off, size, C.byref(ff), C.byref(fb))
        return int(ff.value), int(fb.value)  # WriteStat{FreeWalFid, FreeBytes}

    def index_get(self, ns: bytes, key: bytes):
        f, o, z = C.c_uint64(), C.c_uint64(), C.c_uint64()
        st = lib.oc_bindex_get(self.h, _ptr(ns), len(ns), _ptr(key), len(key), C.byref(f), C.byref(o), C.byref(z))
        return int(st), (int(f.value), int(o.value), int(z.value))

    def put_segment(self, seg, start_off, base_time, ns_size, etag_size, mode, fid, use_rec_fid=False):
        seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
        n = C.c_uint64()
        ec = lib.oc_bindex_put_segment(self.h, _ptr(seg), seg.size, start_off, base_time, ns_size, etag_size, mode,
                                       fid, int(use_rec_fid), C.byref(n))
        return int(ec), int(n.value)

    def compact_filter(self, seg, start_off, base_time, ns_size, etag_size, src_fid, n_rows):
        seg = np.frombuffer(seg, dtype=np.uint8) if isinstance(seg, (bytes, bytearray)) else seg
        keep = np.zeros(max(n_rows, 1), dtype=np.uint8)
        nv = lib.oc_bindex_compact_filter(self.h, _ptr(seg), seg.size, start_off, base_time, ns_size, etag_size,
                                          src_fid, keep.ctypes.data_as(vp), n_rows)
        return keep[:n_rows], int(nv)
