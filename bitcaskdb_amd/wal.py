"""Host-side mirror of the reference's WAL decode interface, backed by the MI355X codec.

Names, argument meaning and error behaviour follow wenzhang-dev/bitcaskDB:
  load_wal            LoadWal / loadSuperBlock            wal.go:218-259, 362-398
  iterate_record      IterateRecord                       record.go:242-266
  iterate_hint        IterateHint                         hint.go:163-188
  compute_crc32       ComputeCRC32                        utils.go:24-29
  compact_one_wal     compactOneWal                       compaction.go:294-327
  new_hint_by_wal     NewHintByWal                        hint.go:123-161
Every record comes out of the GPU decode (libbcw.so); the callback replay below reproduces the
reference's sequential error semantics (records before the first failure are delivered, then
the first error is returned/raised).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


# ---- Go sentinel errors (wal.go:15-26, hint.go:22, record.go:74,147,193) ----
class WalError(Exception):
    pass


class ErrWalMismatchCRC(WalError):
    def __init__(self, msg="CRC mismatch, corrupted data"):
        super().__init__(msg)


class ErrWalUnknownRecordType(WalError):
    def __init__(self, msg="invalid record type"):
        super().__init__(msg)


class ErrWalMismatchSize(WalError):
    def __init__(self, msg="size mismatch, corrupted data"):
        super().__init__(msg)


class ErrWalCorruptedData(WalError):
    def __init__(self, msg="corrupted data"):
        super().__init__(msg)


class ErrWalIncompleteRecord(WalError):
    def __init__(self, msg="incomplete record"):
        super().__init__(msg)


class ErrWalMismatchMagic(WalError):
    def __init__(self, msg="magic number mismatch"):
        super().__init__(msg)


class ErrWalMismatchBlockSize(WalError):
    def __init__(self, msg="block size mismatch"):
        super().__init__(msg)


class ErrInvalidData(WalError):
    def __init__(self, msg="invalid data"):
        super().__init__(msg)


class ErrCorruptedHintRecord(WalError):
    def __init__(self, msg="corrupted hint record"):
        super().__init__(msg)


class RefPanic(WalError):
    """The Go reference panics on these bytes (slice bounds out of range)."""


class ErrShortFile(WalError):
    def __init__(self, msg="EOF"):
        super().__init__(msg)


def compute_crc32(data: bytes) -> int:
    """ComputeCRC32 (utils.go:24-29): masked CRC-32C."""
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data) if data else None
    return int(L.lib.bcw_crc32c_masked(buf, len(data)))


# ---- context ----
class Context:
    """One HIP stream + device tables on one GPU (bcw_ctx)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        rc = L.lib.bcw_ctx_create(device, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"bcw_ctx_create({device}) failed: {L.lib.bcw_strerror(rc).decode()}")
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            L.lib.bcw_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int | None):
        L.lib.bcw_ctx_set_stream(self._h, C.c_void_p(stream_ptr or 0))

    def set_option(self, option: int, value: int):
        """bcw_ctx_set_option (L.OPT_*)"""
        rc = L.lib.bcw_ctx_set_option(self._h, option, value)
        if rc != 0:
            raise ValueError(f"bcw_ctx_set_option({option}, {value}): {L.lib.bcw_strerror(rc).decode()}")

    def sync(self):
        rc = L.lib.bcw_ctx_sync(self._h)
        if rc != 0:
            raise RuntimeError(L.lib.bcw_strerror(rc).decode())

    # synchronous host-in/host-out decode
    def decode(self, seg, start_off: int, base_time: int, ns_size: int, etag_size: int,
               mode: int = L.MODE_RECORD, capacity: int | None = None, with_frags: bool = False):
        seg = np.frombuffer(seg, dtype=np.uint8) if not isinstance(seg, np.ndarray) else seg
        seg = np.ascontiguousarray(seg, dtype=np.uint8)
        n = int(seg.size)
        p = L.DecodeParams(n, base_time, start_off, ns_size, etag_size, mode)
        cap = capacity if capacity is not None else max(16, n // 64)
        while True:
            cols = {name: np.zeros(max(cap, 1), dtype=dt) for name, dt in L.TABLE_COLUMNS}
            tab = L.RecordTable(cap, *[cols[name].ctypes.data_as(getattr(L, "u8p" if dt == "u1" else
                                                                         ("u32p" if dt == "u4" else "u64p")))
                                       for name, dt in L.TABLE_COLUMNS])
            res = L.DecodeResult()
            rc = L.lib.bcw_decode_segment(self._h, seg.ctypes.data_as(C.c_void_p) if n else None, C.byref(p),
                                          C.byref(tab), C.byref(res))
            if rc == L.E_CAPACITY:
                cap = int(res.n_records) + 16
                continue
            if rc != 0:
                raise RuntimeError(f"bcw_decode_segment: {L.lib.bcw_strerror(rc).decode()}")
            break
        nr = int(res.n_records)
        out = Decoded(result=res, table={k: v[:nr].copy() for k, v in cols.items()}, seg=seg, mode=mode,
                      ns_size=ns_size, etag_size=etag_size)
        if with_frags:
            out.frags = self.fragments(max(int(res.n_frags), 1))
        return out

    # synchronous host-in/host-out encode (decode of src + re-encode / hint rebuild on the device)
    def encode(self, src, mode: int, src_start_off: int, dst_base_time: int, fid: int, wal_pos: int, hint_pos: int,
               ns_size: int, etag_size: int, keep=None, wal_cap: int | None = None, hint_cap: int | None = None):
        """Returns (EncodeResult, appended dst WAL bytes, appended hint WAL bytes, rec_off per source row)."""
        src = np.frombuffer(src, dtype=np.uint8) if not isinstance(src, np.ndarray) else src
        src = np.ascontiguousarray(src, dtype=np.uint8)
        n = int(src.size)
        p = L.EncodeParams(n, dst_base_time, fid, wal_pos, hint_pos, src_start_off, mode, ns_size, etag_size)
        keep = np.ascontiguousarray(keep if keep is not None else np.zeros(0), dtype=np.uint8)
        wcap = wal_cap if wal_cap is not None else (n + n // 8 + 4096 if mode == L.ENC_COMPACT else 0)
        hcap = hint_cap if hint_cap is not None else n // 16 + 4096
        nrows = max(16, n // 12 + 16)
        while True:
            wal = np.zeros(max(wcap, 1), dtype=np.uint8)
            hint = np.zeros(max(hcap, 1), dtype=np.uint8)
            offs = np.full(nrows, np.iinfo(np.uint64).max, dtype=np.uint64)
            out = L.EncodeOut(wal.ctypes.data_as(L.u8p), wcap, hint.ctypes.data_as(L.u8p), hcap,
                              offs.ctypes.data_as(L.u64p), nrows)
            res = L.EncodeResult()
            rc = L.lib.bcw_encode_segment(self._h, src.ctypes.data_as(C.c_void_p) if n else None, C.byref(p),
                                          keep.ctypes.data_as(C.c_void_p) if keep.size else None, keep.size,
                                          C.byref(out), C.byref(res))
            if rc == L.E_CAPACITY:
                wcap = max(wcap, int(res.wal_need))
                hcap = max(hcap, int(res.hint_need))
                nrows = max(nrows, int(res.n_in))
                continue
            if rc != 0:
                raise RuntimeError(f"bcw_encode_segment: {L.lib.bcw_strerror(rc).decode()}")
            break
        return res, bytes(wal[:int(res.wal_need)]), bytes(hint[:int(res.hint_need)]), offs[:int(res.n_in)].copy()

    # synchronous batched point reads (Wal.ReadRecord + WalParseRecord + RecordFromBytes per request)
    def read_records(self, seg, offsets, sizes, base_time: int, ns_size: int, etag_size: int, verify: bool = True):
        """Returns (payload bytes per request, rd_status per request, record table dict)."""
        seg = np.ascontiguousarray(np.frombuffer(seg, dtype=np.uint8) if not isinstance(seg, np.ndarray) else seg,
                                   dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
        n = int(offs.size)
        if sizes.size != n:
            raise ValueError("offsets and sizes differ in length")
        p = L.ReadParams(int(seg.size), base_time, ns_size, etag_size, 1 if verify else 0, 0)
        pay = np.zeros(max(int(sizes.sum()), 1), dtype=np.uint8)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        cols = {name: np.zeros(max(n, 1), dtype=dt) for name, dt in L.TABLE_COLUMNS}
        tab = L.RecordTable(n, *[cols[name].ctypes.data_as(getattr(L, "u8p" if dt == "u1" else
                                                                   ("u32p" if dt == "u4" else "u64p")))
                                 for name, dt in L.TABLE_COLUMNS])
        rc = L.lib.bcw_read_records(self._h, seg.ctypes.data_as(C.c_void_p) if seg.size else None, C.byref(p), n,
                                    offs.ctypes.data_as(L.u64p), sizes.ctypes.data_as(L.u64p),
                                    pay.ctypes.data_as(C.c_void_p), st.ctypes.data_as(L.u8p), C.byref(tab))
        if rc != 0:
            raise RuntimeError(f"bcw_read_records: {L.lib.bcw_strerror(rc).decode()}")
        ends = np.concatenate([[0], np.cumsum(sizes, dtype=np.uint64)]) if n else np.zeros(1, np.uint64)
        payloads = [bytes(pay[int(ends[i]):int(ends[i + 1])]) for i in range(n)]
        return payloads, st[:n].copy(), {k: v[:n].copy() for k, v in cols.items()}

    def fragments(self, capacity: int):
        cols = {name: np.zeros(max(capacity, 1), dtype=dt) for name, dt in L.FRAG_COLUMNS}
        ft = L.FragTable(capacity, cols["data_off"].ctypes.data_as(L.u64p), cols["len"].ctypes.data_as(L.u32p),
                         cols["stored_crc"].ctypes.data_as(L.u32p), cols["type"].ctypes.data_as(L.u8p),
                         cols["crc_ok"].ctypes.data_as(L.u8p))
        total = C.c_uint64(0)
        rc = L.lib.bcw_decode_fragments(self._h, C.byref(ft), C.byref(total))
        if rc != 0:
            raise RuntimeError(f"bcw_decode_fragments: {L.lib.bcw_strerror(rc).decode()}")
        t = int(total.value)
        if t > capacity:
            return self.fragments(t)
        return {k: v[:t].copy() for k, v in cols.items()}


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


@dataclass
class Decoded:
    result: L.DecodeResult
    table: dict
    seg: np.ndarray
    mode: int
    ns_size: int
    etag_size: int
    frags: dict | None = None

    @property
    def n_records(self) -> int:
        return int(self.result.n_records)

    def record_bytes(self, r: int) -> bytes:
        """Payload of row r: the data of fragments [first_frag, emit_frag] (needs with_frags)."""
        if self.frags is None:
            raise ValueError("decode(..., with_frags=True) is needed to gather record bytes")
        t, fr = self.table, self.frags
        f0, f1 = int(t["first_frag"][r]), int(t["emit_frag"][r])
        parts = [bytes(self.seg[int(fr["data_off"][g]):int(fr["data_off"][g]) + int(fr["len"][g])])
                 for g in range(f0, f1 + 1)]
        out = b"".join(parts)
        if len(out) != int(t["size"][r]):
            raise AssertionError(f"record {r}: gathered {len(out)} bytes, table says {int(t['size'][r])}")
        return out


# ---- Wal (read side) ----
@dataclass
class Wal:
    data: np.ndarray
    fid: int = 0
    start_off: int = 40
    base_time: int = 0
    create_time: int = 0
    path: str | None = None

    def size(self) -> int:
        return int(self.data.size)

    def BaseTime(self) -> int:  # noqa: N802 (reference spelling)
        return self.base_time


def load_wal(src, fid: int = 0) -> Wal:
    """LoadWal (wal.go:218-259): read the file, validate the super block (CRC, magic, blockSize)."""
    path = None
    if isinstance(src, (str, os.PathLike)):
        path = os.fspath(src)
        with open(path, "rb") as fh:
            raw = fh.read()
    else:
        raw = bytes(src)
    sb = L.SuperBlock()
    buf = (C.c_uint8 * max(len(raw), 1)).from_buffer_copy(raw if raw else b"\0")
    rc = L.lib.bcw_load_super_block(buf, len(raw), C.byref(sb))
    if rc == L.SB_SHORT:
        raise ErrShortFile()
    if rc == L.SB_CRC:
        raise ErrWalMismatchCRC()
    if rc == L.SB_MAGIC:
        raise ErrWalMismatchMagic()
    if rc == L.SB_BLOCKSIZE:
        raise ErrWalMismatchBlockSize()
    return Wal(np.frombuffer(raw, dtype=np.uint8), fid, int(sb.start_off), int(sb.base_time),
               int(sb.create_time), path)


# ---- records ----
@dataclass
class Meta:
    expire: int = 0
    etag: bytes | None = None
    flags: int = 0
    app_meta: bytes = b""  # msgpack bytes, opaque (msgpack parity unpinned)

    def is_tombstone(self) -> bool:
        return bool(self.flags & 1)


@dataclass
class Record:
    ns: bytes
    key: bytes
    value: bytes
    meta: Meta = field(default_factory=Meta)


@dataclass
class HintRecord:
    ns: bytes
    key: bytes
    fid: int
    off: int
    size: int


def _frag_error(res):
    if res.err_class == L.ERR_CRC:
        return ErrWalMismatchCRC()
    if res.err_class == L.ERR_TYPE:
        return ErrWalUnknownRecordType()
    if res.err_class == L.ERR_PANIC:
        return RefPanic("slice bounds out of range (startOff beyond file size)")
    if res.err_class == L.ERR_INTERNAL:
        raise RuntimeError("bcw decode: a device-side wait exceeded its bound or the fragment table disagreed with the "
                           "chunk stream (protocol failure); no row was delivered")
    return None


def _record_of(dec: Decoded, r: int, payload: bytes) -> Record:
    t = dec.table
    flags = int(t["flags"][r])
    o = int(t["etag_off"][r])
    etag_len = 0 if flags & 1 else dec.etag_size
    hdr = int(t["hdr_size"][r])
    kl, vl, ml = int(t["key_len"][r]), int(t["val_len"][r]), int(t["meta_len"][r])
    key = payload[hdr:hdr + kl]
    value = payload[hdr + kl:hdr + kl + vl]
    meta = payload[hdr + kl + vl:hdr + kl + vl + ml]
    return Record(ns=payload[1:1 + dec.ns_size], key=key, value=value,
                  meta=Meta(expire=int(t["expire"][r]), etag=payload[o:o + etag_len],
                            flags=1 if flags & 4 else 0, app_meta=meta))


def iterate_record(wal: Wal, cb, ns_size: int = 20, etag_size: int = 20, ctx: Context | None = None):
    """IterateRecord (record.go:242-266): cb(record, foff, size) per record; raises the first error."""
    ctx = ctx or default_context()
    dec = ctx.decode(wal.data, wal.start_off, wal.base_time, ns_size, etag_size, L.MODE_RECORD, with_frags=True)
    if dec.result.err_class == L.ERR_INTERNAL:  # before any row reaches the callback
        _frag_error(dec.result)
    for r in range(dec.n_records):
        st = int(dec.table["status"][r])
        if st == L.ST_INVALID:
            raise ErrInvalidData()
        if st == L.ST_PANIC:
            raise RefPanic("slice bounds out of range")
        if st == L.ST_UNSUPPORTED:
            raise WalError("record length >= 2^32 is not supported by the device table")
        payload = dec.record_bytes(r)
        ret = cb(_record_of(dec, r, payload), int(dec.table["foff"][r]), int(dec.table["size"][r]))
        if ret is not None:
            raise ret if isinstance(ret, BaseException) else WalError(str(ret))
    err = _frag_error(dec.result)
    if err is not None:
        raise err


def iterate_hint(hint: Wal, cb, ns_size: int = 20, ctx: Context | None = None):
    """IterateHint (hint.go:163-188): cb(HintRecord) per record; raises the first error."""
    ctx = ctx or default_context()
    dec = ctx.decode(hint.data, hint.start_off, hint.base_time, ns_size, 0, L.MODE_HINT, with_frags=True)
    if dec.result.err_class == L.ERR_INTERNAL:  # before any row reaches the callback
        _frag_error(dec.result)
    for r in range(dec.n_records):
        st = int(dec.table["status"][r])
        if st == L.ST_INVALID:
            raise ErrCorruptedHintRecord()
        if st == L.ST_PANIC:
            raise RefPanic("slice bounds out of range")
        payload = dec.record_bytes(r)
        # key offset = NsSize + len(uvarint keyLen) (hint.go:62-66); the table's u8 hdr_size holds it mod 256
        ko = ns_size + 1
        while ko - ns_size < 10 and payload[ko - 1] & 0x80:
            ko += 1
        kl = int(dec.table["key_len"][r])
        rec = HintRecord(ns=payload[:ns_size], key=payload[ko:ko + kl], fid=int(dec.table["expire"][r]),
                         off=int(dec.table["aux0"][r]), size=int(dec.table["aux1"][r]))
        ret = cb(rec)
        if ret is not None:
            raise ret if isinstance(ret, BaseException) else WalError(str(ret))
    err = _frag_error(dec.result)
    if err is not None:
        raise err


_RD_ERRORS = {
    L.RD_BEYOND: lambda: WalError("read beyond file size"),
    L.RD_CORRUPTED: lambda: ErrWalCorruptedData(),
    L.RD_CRC: lambda: ErrWalMismatchCRC(),
    L.RD_SIZE: lambda: ErrWalMismatchSize(),
    L.RD_TYPE: lambda: ErrWalUnknownRecordType(),
    L.RD_INCOMPLETE: lambda: ErrWalIncompleteRecord(),
    L.RD_PANIC: lambda: RefPanic("slice bounds out of range (zero-size read)"),
}


def read_records(wal: Wal, offsets, sizes, verify: bool = True, ns_size: int = 20, etag_size: int = 20,
                 ctx: Context | None = None) -> list:
    """The record fetch of DBImpl.Get / GetV2 (db_impl.go:567-631) for many index values at once:
    Wal.ReadRecord(off, size, verifyChecksum) (wal.go:556-573) then RecordFromBytes (record.go:140-239).
    One entry per request: a Record, or the exception the reference returns for it (not raised)."""
    ctx = ctx or default_context()
    pays, st, t = ctx.read_records(wal.data, offsets, sizes, wal.base_time, ns_size, etag_size, verify)
    view = Decoded(result=L.DecodeResult(), table=t, seg=wal.data, mode=L.MODE_RECORD, ns_size=ns_size,
                   etag_size=etag_size)
    out = []
    for i, payload in enumerate(pays):
        if st[i] != L.RD_OK:
            out.append(_RD_ERRORS[int(st[i])]())
        elif t["status"][i] == L.ST_INVALID:
            out.append(ErrInvalidData())
        elif t["status"][i] == L.ST_PANIC:
            out.append(RefPanic("slice bounds out of range"))
        else:
            out.append(_record_of(view, i, payload))
    return out


# ---- write side: compaction re-encode and hint rebuild ----
class WalFile:
    """In-memory WAL file being written (NewWal + WriteRecord appends, wal.go:262-360, 490-553)."""

    def __init__(self, fid: int, base_time: int, create_time: int | None = None):
        sb = (C.c_uint8 * 40)()
        L.lib.bcw_write_super_block(sb, create_time if create_time is not None else base_time, base_time)
        self.data = bytearray(bytes(sb))
        self.fid = fid
        self.base_time = base_time

    def size(self) -> int:
        return len(self.data)

    def BaseTime(self) -> int:  # noqa: N802
        return self.base_time

    def Fid(self) -> int:  # noqa: N802
        return self.fid

    def as_wal(self) -> Wal:
        return load_wal(bytes(self.data), self.fid)


_ENC_ERRORS = {L.ENC_ERR_EXPIRE: lambda: WalError("invalid expire"),
               L.ENC_ERR_PANIC: lambda: RefPanic("index out of range (PutUvarint into [MaxVarintLen32]byte)"),
               # nothing was appended: the encode's own decode of the source delivered no usable table (it reported
               # BCW_ERR_INTERNAL, or its table is smaller than the decode), or another decode ran on the context in
               # between. A compaction must not report success here: the caller would drop the source with no copy.
               L.ENC_ERR_TABLE: lambda: RuntimeError("bcw encode: the source decode delivered no usable record table "
                                                     "(BCW_ENC_ERR_TABLE); nothing was written"),
               L.ENC_ERR_STALE: lambda: RuntimeError("bcw encode: the source decode is not the context's latest "
                                                     "(BCW_ENC_ERR_STALE); nothing was written")}


def _src_error(res, dec_class, status):
    if status == L.ST_INVALID:
        return ErrInvalidData()
    if status == L.ST_PANIC:
        return RefPanic("slice bounds out of range")
    if status == L.ST_UNSUPPORTED:
        return WalError("record length >= 2^32 is not supported by the device table")
    return _frag_error(type("R", (), {"err_class": dec_class})())


def _encode_fails(expire: int, dst_base: int) -> bool:
    """Record.Encode (record.go:63-78) fails on this row: "invalid expire" or the 5-byte varint panic."""
    return expire != 0 and (expire < dst_base or expire - dst_base >= 1 << 35)


def _filter_rows(src: Wal, flt, dst_base: int, ns_size: int, etag_size: int, ctx: Context) -> np.ndarray:
    """The keep mask of compactOneWal's loop (compaction.go:299-311) with a doFilter callback, called in
    record order exactly as the reference calls it: not for rows at or after the first row
    RecordFromBytes rejects, and not after the first kept row whose Record.Encode fails."""
    dec = ctx.decode(src.data, src.start_off, src.base_time, ns_size, etag_size, L.MODE_RECORD, with_frags=True)
    t = dec.table
    rows = []
    for r in range(dec.n_records):
        if int(t["status"][r]) != L.ST_OK:
            break
        rec = _record_of(dec, r, dec.record_bytes(r))
        k = not flt(rec, src.fid, int(t["foff"][r]) - HEADER)
        rows.append(k)
        if k and _encode_fails(int(t["expire"][r]), dst_base):
            break
    return np.array(rows, dtype=np.uint8)


def compact_one_wal(dst: WalFile, hint: WalFile, src: Wal, keep, ns_size: int = 20, etag_size: int = 20,
                    ctx: Context | None = None):
    """compactOneWal (compaction.go:294-327): every delivered source record with keep[i] (the doFilter
    verdict, compaction.go:303) is re-encoded against dst's baseTime and appended to dst, its hint to
    `hint`. Returns the dst offsets per source row (2**64-1: not written). Raises the reference's error
    after appending what the reference appends before it."""
    ctx = ctx or default_context()
    if callable(keep):  # doFilter(record, fid, off) -> True drops the record (compaction.go:329-348)
        keep = _filter_rows(src, keep, dst.base_time, ns_size, etag_size, ctx)
    res, wal, hb, offs = ctx.encode(src.data, L.ENC_COMPACT, src.start_off, dst.base_time, dst.fid, dst.size(),
                                    hint.size(), ns_size, etag_size, keep)
    dst.data += wal
    hint.data += hb
    if res.err_class == L.ENC_ERR_SRC:
        st = L.ST_OK
        if res.err_record >= 0:
            dec = ctx.decode(src.data, src.start_off, src.base_time, ns_size, etag_size)
            st = int(dec.table["status"][res.err_record])
        raise _src_error(res, res.src_err_class, st)
    if res.err_class in _ENC_ERRORS:
        raise _ENC_ERRORS[res.err_class]()
    return offs


def new_hint_by_wal(wal: Wal, ns_size: int = 20, etag_size: int = 20, ctx: Context | None = None,
                    create_time: int | None = None) -> WalFile:
    """NewHintByWal (hint.go:123-161): the hint WAL (same fid and baseTime) of a data WAL."""
    ctx = ctx or default_context()
    h = WalFile(wal.fid, wal.base_time, create_time)
    res, _, hb, _ = ctx.encode(wal.data, L.ENC_HINT, wal.start_off, wal.base_time, wal.fid, 40, h.size(), ns_size,
                               etag_size)
    h.data += hb
    if res.err_class == L.ENC_ERR_SRC:
        st = L.ST_OK
        if res.err_record >= 0:
            dec = ctx.decode(wal.data, wal.start_off, wal.base_time, ns_size, etag_size)
            st = int(dec.table["status"][res.err_record])
        raise _src_error(res, res.src_err_class, st)
    if res.err_class in _ENC_ERRORS:
        raise _ENC_ERRORS[res.err_class]()
    return h


HEADER = L.HEADER_SIZE
