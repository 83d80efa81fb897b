"""Host-side mirror of the reference index interface, backed by the device index of libbcw.so.

Names, argument meaning and error behaviour follow wenzhang-dev/bitcaskDB:
  Index.get / put / delete / soft_delete   Index.Get/Put/Delete/SoftDelete   index.go:81-165
  murmur3_sum64                            IndexOperator.Hash                index.go:15-19
  recover_from_wals                        DBImpl.recoverFromWals / recoverFromWal  db_impl.go:268-314
  compact_one_wal_filtered                 compactOneWal with doFilter       compaction.go:294-348
The index lives in HBM (bcw_index); every operation goes through the C-ABI, there is no host fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .wal import (Context, Wal, WalError, WalFile, _ENC_ERRORS, _frag_error, _src_error, default_context)


class ErrKeyNotFound(WalError):
    def __init__(self, msg="key not found"):  # db.go:33
        super().__init__(msg)


class ErrKeySoftDeleted(WalError):
    def __init__(self, msg="key soft delete"):  # db.go:35
        super().__init__(msg)


def merged_key(ns: bytes, key: bytes) -> bytes:
    """MergedKey (utils.go:133-139)."""
    return bytes(ns) + bytes(key)


def murmur3_sum64(data: bytes) -> int:
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    return int(L.lib.bcw_murmur3_sum64(buf, len(data)))


def _pack(keys):
    off = np.zeros(len(keys) + 1, dtype=np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    flat = np.frombuffer(b"".join(keys), dtype=np.uint8) if off[-1] else np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(flat), off


@dataclass
class IndexStats:
    live: int
    slots_used: int
    slot_capacity: int
    arena_used: int
    arena_capacity: int
    overflow: int
    limited: int = 0
    evicted: int = 0
    evicted_bytes: int = 0


class Index:
    """The device index (bcw_index) bound to one Context."""

    def __init__(self, ctx: Context | None = None, keys: int = 1 << 16, arena_bytes: int = 8 << 20):
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        rc = L.lib.bcw_index_create(self.ctx.handle, keys, arena_bytes, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"bcw_index_create: {L.lib.bcw_strerror(rc).decode()}")
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            L.lib.bcw_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- batches (DBImpl.writeIndex, db_impl.go:433-452) ----
    def apply(self, ops, keys, fid=None, off=None, size=None, stats: bool = False):
        """ops[i] in (IDX_PUT, IDX_DELETE, IDX_SOFT_DELETE) on merged key keys[i], applied in order.
        stats: also return every op's WriteStat (index.go:100-165) as (found, free_fid, free_bytes) arrays."""
        n = len(keys)
        if n == 0:
            return (np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint64)) if stats else None
        flat, koff = _pack(keys)
        ops = np.ascontiguousarray(ops, dtype=np.uint8)
        z = np.zeros(n, dtype=np.uint64)
        fid = np.ascontiguousarray(fid if fid is not None else z, dtype=np.uint64)
        off = np.ascontiguousarray(off if off is not None else z, dtype=np.uint64)
        size = np.ascontiguousarray(size if size is not None else z, dtype=np.uint64)
        found, ffid, fbytes = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
        rc = L.lib.bcw_index_apply_stat(self._h, n, flat.ctypes.data_as(C.c_void_p), koff.ctypes.data_as(L.u64p),
                                        ops.ctypes.data_as(L.u8p), fid.ctypes.data_as(L.u64p),
                                        off.ctypes.data_as(L.u64p), size.ctypes.data_as(L.u64p),
                                        found.ctypes.data_as(L.u8p) if stats else None,
                                        ffid.ctypes.data_as(L.u64p) if stats else None,
                                        fbytes.ctypes.data_as(L.u64p) if stats else None)
        if rc != 0:
            raise RuntimeError(f"bcw_index_apply: {L.lib.bcw_strerror(rc).decode()}")
        return (found, ffid, fbytes) if stats else None

    def write_index(self, ops, keys, fid=None, off=None, size=None) -> dict:
        """DBImpl.writeIndex (db_impl.go:433-452): apply the batch, return writeStats {FreeWalFid: FreeBytes}
        (a not-found Delete adds 0 to fid 0, as the reference's zero WriteStat does)."""
        found, ffid, fbytes = self.apply(ops, keys, fid, off, size, stats=True)
        out: dict = {}
        for f, b in zip(ffid.tolist(), fbytes.tolist()):
            out[f] = out.get(f, 0) + b
        return out

    def clear(self):
        """remove every key (capacity kept): with apply() of a Go index's live entries, a snapshot load"""
        rc = L.lib.bcw_index_clear(self._h)
        if rc != 0:
            raise RuntimeError(f"bcw_index_clear: {L.lib.bcw_strerror(rc).decode()}")

    def load_snapshot(self, entries: dict):
        """make the device index hold exactly `entries` ({merged key: (fid, off, size)}, e.g. the live entries of
        a bounded, evicting Go index at compaction start), for the device doFilter"""
        self.clear()
        keys = list(entries)
        vals = np.array([entries[k] for k in keys], dtype=np.uint64).reshape(-1, 3)
        self.apply([L.IDX_PUT] * len(keys), keys, vals[:, 0], vals[:, 1], vals[:, 2])

    def get_many(self, keys):
        """Index.Get of merged keys: (status, fid, off, size) arrays; status IDX_*."""
        n = len(keys)
        st = np.zeros(max(n, 1), dtype=np.uint8)
        fid, off, size = (np.zeros(max(n, 1), dtype=np.uint64) for _ in range(3))
        if n:
            flat, koff = _pack(keys)
            rc = L.lib.bcw_index_get(self._h, n, flat.ctypes.data_as(C.c_void_p), koff.ctypes.data_as(L.u64p),
                                     fid.ctypes.data_as(L.u64p), off.ctypes.data_as(L.u64p),
                                     size.ctypes.data_as(L.u64p), st.ctypes.data_as(L.u8p))
            if rc != 0:
                raise RuntimeError(f"bcw_index_get: {L.lib.bcw_strerror(rc).decode()}")
        return st[:n], fid[:n], off[:n], size[:n]

    # ---- the reference's single-key interface (index.go:81-165) ----
    def put(self, ns: bytes, key: bytes, fid: int, off: int, sz: int):
        self.apply([L.IDX_PUT], [merged_key(ns, key)], [fid], [off], [sz])

    def delete(self, ns: bytes, key: bytes):
        self.apply([L.IDX_DELETE], [merged_key(ns, key)])

    def soft_delete(self, ns: bytes, key: bytes):
        self.apply([L.IDX_SOFT_DELETE], [merged_key(ns, key)])

    def get(self, ns: bytes, key: bytes):
        """(fid, off, sz); raises ErrKeyNotFound / ErrKeySoftDeleted as index.go:81-98."""
        st, fid, off, size = self.get_many([merged_key(ns, key)])
        if st[0] == L.IDX_NOT_FOUND:
            raise ErrKeyNotFound()
        if st[0] == L.IDX_SOFT_DELETED:
            raise ErrKeySoftDeleted()
        return int(fid[0]), int(off[0]), int(size[0])

    def stats(self) -> IndexStats:
        info = L.IndexInfo()
        rc = L.lib.bcw_index_stats(self._h, C.byref(info))
        if rc != 0:
            raise RuntimeError(f"bcw_index_stats: {L.lib.bcw_strerror(rc).decode()}")
        return IndexStats(int(info.live), int(info.slots_used), int(info.slot_capacity), int(info.arena_used),
                          int(info.arena_capacity), int(info.overflow), int(info.limited), int(info.evicted),
                          int(info.evicted_bytes))

    def set_limit(self, limited: int):
        """IndexLimited (db.go:71): at most `limited` keys, 16 shards of limited / 16 (map.go's ShardMap), least
        recently set entries evicted after every batch (bcw_index_set_limit: the deterministic stand-in for the
        reference's Rand-sampled eviction, map.go:395-420). 0: unbounded."""
        rc = L.lib.bcw_index_set_limit(self._h, limited)
        if rc != 0:
            raise RuntimeError(f"bcw_index_set_limit: {L.lib.bcw_strerror(rc).decode()}")

    def export(self, fids=None) -> dict:
        """every live entry: {merged key: (fid, off, size)}; fids: only entries whose value fid is one of them
        (bcw_index_export_fids)"""
        fa = np.ascontiguousarray(sorted(set(fids)) if fids is not None else [], dtype=np.uint64)
        nf = int(fa.size)
        fp = fa.ctypes.data_as(L.u64p) if nf else None
        if fids is not None and nf == 0:
            return {}
        n, kb = C.c_uint64(), C.c_uint64()
        rc = L.lib.bcw_index_export_fids(self._h, fp, nf, None, 0, None, None, None, None, 0, C.byref(n),
                                         C.byref(kb))
        if rc not in (0, L.E_CAPACITY):
            raise RuntimeError(f"bcw_index_export: {L.lib.bcw_strerror(rc).decode()}")
        if n.value == 0:
            return {}
        cap, kcap = int(n.value), int(kb.value)
        keys = np.zeros(max(kcap, 1), dtype=np.uint8)
        koff = np.zeros(cap + 1, dtype=np.uint64)
        fid, off, size = (np.zeros(cap, dtype=np.uint64) for _ in range(3))
        rc = L.lib.bcw_index_export_fids(self._h, fp, nf, keys.ctypes.data_as(C.c_void_p), kcap,
                                         koff.ctypes.data_as(L.u64p), fid.ctypes.data_as(L.u64p),
                                         off.ctypes.data_as(L.u64p), size.ctypes.data_as(L.u64p), cap, C.byref(n),
                                         C.byref(kb))
        if rc != 0:
            raise RuntimeError(f"bcw_index_export: {L.lib.bcw_strerror(rc).decode()}")
        kbytes = keys.tobytes()
        return {kbytes[int(koff[i]):int(koff[i + 1])]: (int(fid[i]), int(off[i]), int(size[i])) for i in range(cap)}

    # ---- table-driven (device-resident) Put loops ----
    def recover_segment(self, data, mode: int, fid: int, start_off: int, base_time: int, ns_size: int,
                        etag_size: int, use_record_fid: bool = False):
        """One recoverFromWal iteration (db_impl.go:290-313): returns (DecodeResult, IndexResult)."""
        seg = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data)
        p = L.DecodeParams(seg.size, base_time, start_off, ns_size, etag_size, mode)
        dres, ires = L.DecodeResult(), L.IndexResult()
        rc = L.lib.bcw_index_recover_segment(self.ctx.handle, self._h, seg.ctypes.data_as(C.c_void_p) if seg.size
                                             else None, C.byref(p), fid, int(use_record_fid), C.byref(dres),
                                             C.byref(ires))
        if rc != 0:
            raise RuntimeError(f"bcw_index_recover_segment: {L.lib.bcw_strerror(rc).decode()}")
        return dres, ires


def _iteration_error(dres, ires, hint: bool):
    """the error IterateRecord / IterateHint returns after the delivered rows (record.go:246-263)."""
    if ires.n_in < dres.n_records:  # a rejected row stops the iteration
        return WalError("corrupted hint record") if hint else WalError("invalid data")
    return _frag_error(dres)


def recover_from_wals(index: Index, files, ns_size: int = 20, etag_size: int = 20, contexts=None):
    """recoverFromWals (db_impl.go:268-314): for every fid in ascending order, Put every record of its hint
    file (IterateHint); if that iteration fails, Put every record of the data WAL (IterateRecord), keeping
    the puts already applied. files: {fid: (Wal data, Wal hint or None)}. Raises the data WAL's error.
    contexts (a list of Context, any devices): the files are decoded concurrently, round-robin over them, and
    the index still receives each file's puts in ascending fid (bcw_recover_wals)."""
    if contexts:
        return _recover_fanout(index, files, ns_size, etag_size, contexts)
    for fid in sorted(files):
        wal, hint = files[fid]
        if hint is not None:
            dres, ires = index.recover_segment(hint.data, L.MODE_HINT, fid, hint.start_off, hint.base_time, ns_size,
                                               0)
            if ires.err_class:
                raise RuntimeError(f"index put failed: {ires.err_class}")
            if _iteration_error(dres, ires, True) is None:
                continue
        dres, ires = index.recover_segment(wal.data, L.MODE_RECORD, fid, wal.start_off, wal.base_time, ns_size,
                                           etag_size)
        if ires.err_class:
            raise RuntimeError(f"index put failed: {ires.err_class}")
        err = _iteration_error(dres, ires, False)
        if err is not None:
            raise err


_NUL = np.zeros(1, dtype=np.uint8)


def _ctx_array(contexts):
    arr = (C.c_void_p * len(contexts))(*[c.handle for c in contexts])
    return arr, len(contexts)


def _recover_fanout(index: Index, files, ns_size: int, etag_size: int, contexts):
    fids = sorted(files)
    keep = []  # the segments stay referenced for the call
    arr = (L.RecoverFile * max(len(fids), 1))()
    for k, fid in enumerate(fids):
        wal, hint = files[fid]
        w = np.ascontiguousarray(wal.data)
        keep.append(w)
        arr[k].fid = fid
        arr[k].wal = w.ctypes.data if w.size else None
        arr[k].wal_p = L.DecodeParams(w.size, wal.base_time, wal.start_off, ns_size, etag_size, L.MODE_RECORD)
        if hint is not None:
            h = np.ascontiguousarray(hint.data)
            keep.append(h)
            arr[k].hint = h.ctypes.data if h.size else _NUL.ctypes.data  # present, even when empty
            arr[k].hint_p = L.DecodeParams(h.size, hint.base_time, hint.start_off, ns_size, 0, L.MODE_HINT)
        else:
            arr[k].hint = None
            arr[k].hint_p = L.DecodeParams(0, 0, 0, ns_size, 0, L.MODE_HINT)
    st = (L.RecoverStatus * max(len(fids), 1))()
    stop = C.c_int64(-1)
    ctxs, n_ctx = _ctx_array(contexts)
    rc = L.lib.bcw_recover_wals(index.handle, ctxs, n_ctx, arr, len(fids), st, C.byref(stop))
    if rc != 0:
        raise RuntimeError(f"bcw_recover_wals: {L.lib.bcw_strerror(rc).decode()}")
    if stop.value < 0:
        return
    s = st[stop.value]
    if s.rc != 0:
        raise RuntimeError(f"bcw_recover_wals (fid {fids[stop.value]}): {L.lib.bcw_strerror(s.rc).decode()}")
    if s.used in (L.RECOVER_HINT, L.RECOVER_HINT_WAL) and s.hint_ires.err_class:
        raise RuntimeError(f"index put failed: {s.hint_ires.err_class}")
    if s.used == L.RECOVER_HINT:  # the hint decode gave up (BCW_ERR_INTERNAL): raises
        _iteration_error(s.hint_dres, s.hint_ires, True)
        raise RuntimeError("bcw_recover_wals: stopped at a hint without an error")
    if s.wal_ires.err_class:
        raise RuntimeError(f"index put failed: {s.wal_ires.err_class}")
    err = _iteration_error(s.wal_dres, s.wal_ires, False)
    if err is not None:
        raise err


def compact_wals_filtered(dst: WalFile, hint: WalFile, srcs, index: Index, ns_size: int = 20, etag_size: int = 20,
                          contexts=None):
    """doCompactionWork's loop (compaction.go:201-211): compact_one_wal_filtered of every source Wal in order
    into one dst / hint pair. contexts (a list of Context, any devices): the sources are uploaded, decoded and
    filtered concurrently, round-robin over them; the encodes append in source order (bcw_compact_wals).
    Returns [(dst offsets per source row, rows kept)] per source; raises the first source's error after the
    appends the reference makes before it."""
    if not contexts:
        return [compact_one_wal_filtered(dst, hint, s, index, ns_size, etag_size) for s in srcs]
    out = []
    k0 = 0
    caps = {}
    while k0 < len(srcs):
        part = srcs[k0:]
        n = len(part)
        arr = (L.CompactSrc * n)()
        keep = []
        bufs = []
        for k, src in enumerate(part):
            seg = np.ascontiguousarray(src.data)
            m = int(seg.size)
            wcap, hcap, nrows = caps.get(k0 + k, (m + m // 8 + 4096, m // 16 + 4096, max(16, m // 12 + 16)))
            wal = np.zeros(max(wcap, 1), dtype=np.uint8)
            hb = np.zeros(max(hcap, 1), dtype=np.uint8)
            offs = np.full(nrows, np.iinfo(np.uint64).max, dtype=np.uint64)
            keep.append(seg)
            bufs.append((wal, hb, offs))
            arr[k].fid = src.fid
            arr[k].data = seg.ctypes.data if m else None
            arr[k].len = m
            arr[k].start_off = src.start_off
            arr[k].out = L.EncodeOut(wal.ctypes.data_as(L.u8p), wcap, hb.ctypes.data_as(L.u8p), hcap,
                                     offs.ctypes.data_as(L.u64p), nrows)
        p = L.EncodeParams(0, dst.base_time, dst.fid, dst.size(), hint.size(), 0, L.ENC_COMPACT, ns_size, etag_size)
        res = (L.EncodeResult * n)()
        filt = (L.IndexResult * n)()
        done = C.c_uint64(0)
        ctxs, n_ctx = _ctx_array(contexts)
        rc = L.lib.bcw_compact_wals(index.handle, ctxs, n_ctx, arr, n, C.byref(p), res, filt, C.byref(done))
        for k in range(int(done.value)):
            r, (wal, hb, offs) = res[k], bufs[k]
            dst.data += wal[:int(r.wal_need)].tobytes()
            hint.data += hb[:int(r.hint_need)].tobytes()
            out.append((offs[:int(r.n_in)].copy(), int(filt[k].n_done)))
        if rc == L.E_CAPACITY:
            k = int(done.value)
            r, m = res[k], int(part[k].data.size)
            wcap, hcap, nrows = caps.get(k0 + k, (m + m // 8 + 4096, m // 16 + 4096, max(16, m // 12 + 16)))
            grown = (max(wcap, int(r.wal_need)), max(hcap, int(r.hint_need)), max(nrows, int(r.n_in)))
            if grown == (wcap, hcap, nrows):  # not an output shortfall (a staging or fragment capacity refusal)
                raise RuntimeError(f"bcw_compact_wals: {L.lib.bcw_strerror(rc).decode()}")
            caps[k0 + k] = grown
            k0 += k
            continue
        if rc != 0:
            raise RuntimeError(f"bcw_compact_wals: {L.lib.bcw_strerror(rc).decode()}")
        if done.value:
            r = res[int(done.value) - 1]
            src = part[int(done.value) - 1]
            if r.err_class == L.ENC_ERR_SRC:
                st = L.ST_OK
                if r.err_record >= 0:
                    dec = index.ctx.decode(src.data, src.start_off, src.base_time, ns_size, etag_size)
                    st = int(dec.table["status"][r.err_record])
                raise _src_error(r, r.src_err_class, st)
            if r.err_class in _ENC_ERRORS:
                raise _ENC_ERRORS[r.err_class]()
        break
    return out


def compact_one_wal_filtered(dst: WalFile, hint: WalFile, src: Wal, index: Index, ns_size: int = 20,
                             etag_size: int = 20, ctx: Context | None = None):
    """compactOneWal (compaction.go:294-327) with doFilter (compaction.go:329-348, no user CompactionFilter)
    evaluated on the device against `index`: decode -> filter -> re-encode in one device pass. Returns
    (dst offsets per source row, rows kept); raises the reference's error after appending what the
    reference appends before it."""
    ctx = ctx or index.ctx
    seg = np.ascontiguousarray(src.data)
    n = int(seg.size)
    p = L.EncodeParams(n, dst.base_time, dst.fid, dst.size(), hint.size(), src.start_off, L.ENC_COMPACT, ns_size,
                       etag_size)
    wcap, hcap, nrows = n + n // 8 + 4096, n // 16 + 4096, max(16, n // 12 + 16)
    while True:
        wal = np.zeros(max(wcap, 1), dtype=np.uint8)
        hb = np.zeros(max(hcap, 1), dtype=np.uint8)
        offs = np.full(nrows, np.iinfo(np.uint64).max, dtype=np.uint64)
        out = L.EncodeOut(wal.ctypes.data_as(L.u8p), wcap, hb.ctypes.data_as(L.u8p), hcap, offs.ctypes.data_as(L.u64p),
                          nrows)
        res, fres = L.EncodeResult(), L.IndexResult()
        rc = L.lib.bcw_compact_segment(ctx.handle, index.handle, seg.ctypes.data_as(C.c_void_p) if n else None,
                                       C.byref(p), src.fid, C.byref(out), C.byref(res), C.byref(fres))
        if rc == L.E_CAPACITY:
            grown = (max(wcap, int(res.wal_need)), max(hcap, int(res.hint_need)), max(nrows, int(res.n_in)))
            if grown == (wcap, hcap, nrows):  # not an output shortfall (a staging or fragment capacity refusal)
                raise RuntimeError(f"bcw_compact_segment: {L.lib.bcw_strerror(rc).decode()}")
            wcap, hcap, nrows = grown
            continue
        if rc != 0:
            raise RuntimeError(f"bcw_compact_segment: {L.lib.bcw_strerror(rc).decode()}")
        break
    dst.data += wal[:int(res.wal_need)].tobytes()
    hint.data += hb[:int(res.hint_need)].tobytes()
    if res.err_class == L.ENC_ERR_SRC:
        st = L.ST_OK
        if res.err_record >= 0:
            dec = ctx.decode(src.data, src.start_off, src.base_time, ns_size, etag_size)
            st = int(dec.table["status"][res.err_record])
        raise _src_error(res, res.src_err_class, st)
    if res.err_class in _ENC_ERRORS:
        raise _ENC_ERRORS[res.err_class]()
    return offs[:int(res.n_in)].copy(), int(fres.n_done)
