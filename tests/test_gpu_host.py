"""GPU tests of the host-side mirror (bitcaskdb_amd/wal.py: the IterateRecord / IterateHint callback
replay, compactOneWal with a doFilter callback, NewHintByWal) and of the C-ABI's boundary contract
(decode generations, table capacity, rec_off capacity, two contexts used from two threads at once)."""
from __future__ import annotations

import ctypes as C
import random
import threading

import numpy as np
import pytest

import _oracle as O
import cases
from bitcaskdb_amd import _lib as L
from bitcaskdb_amd import wal as W

pytestmark = pytest.mark.gpu
BASE = cases.BASE


def oracle_records(data, ns=20, etag=20, base=BASE):
    d = O.decode(data, 40, base, ns, etag)
    return d


def mixed_wal(seed, n=300, bad_row=None):
    rng = random.Random(seed)
    payloads = []
    for i in range(n):
        etag = bytes(rng.getrandbits(8) for _ in range(20)) if rng.random() < 0.3 else b""
        expire = BASE + rng.choice([0, 5, 1000]) if rng.random() < 0.3 else 0
        meta = b"\x81\xa3foo\xa3bar" if rng.random() < 0.1 else b""
        payloads.append(cases.rec(i, vlen=rng.choice([0, 10, 4096, 40000]), etag=etag, expire=expire,
                                  tomb=rng.random() < 0.1, meta=meta))
    if bad_row is not None:
        payloads[bad_row] = b"\x05garbage-bytes"
    data, offs = cases.wal_of(payloads)
    return data, payloads, offs


def test_iterate_record_replay(ctx):
    data, payloads, offs = mixed_wal(1)
    wal = W.load_wal(data, fid=4)
    got = []
    W.iterate_record(wal, lambda r, foff, size: got.append((r, foff, size)), 20, 20, ctx)
    ref = oracle_records(data)
    assert len(got) == len(ref.recs) == len(payloads)
    for i, (r, foff, size) in enumerate(got):
        rr = ref.recs[i]
        assert foff == rr["foff"] and size == rr["size"] == len(payloads[i])
        assert foff - 7 == offs[i]
        p = ref.payloads[i]
        h = int(rr["hdr_size"])
        assert r.ns == p[1:21]
        assert r.key == p[h:h + int(rr["key_len"])]
        assert r.value == p[h + int(rr["key_len"]):h + int(rr["key_len"]) + int(rr["val_len"])]
        assert r.meta.expire == int(rr["expire"])
        assert r.meta.is_tombstone() == bool(rr["flags"] & 4)


def test_iterate_record_error_replay(ctx):
    # a RecordFromBytes failure: rows before it are delivered, then "invalid data"
    data, _, _ = mixed_wal(2, bad_row=120)
    got = []
    with pytest.raises(W.ErrInvalidData):
        W.iterate_record(W.load_wal(data), lambda r, f, s: got.append(f), 20, 20, ctx)
    assert len(got) == 120
    # a CRC failure: every record before the failing fragment is delivered, then ErrWalMismatchCRC
    data, _, offs = mixed_wal(3)
    bad = bytearray(data)
    bad[offs[200] + 7 + 3] ^= 0x01
    ref = oracle_records(bytes(bad))
    got = []
    with pytest.raises(W.ErrWalMismatchCRC):
        W.iterate_record(W.load_wal(bytes(bad)), lambda r, f, s: got.append(f), 20, 20, ctx)
    assert got == [int(x) for x in ref.recs["foff"]] and len(got) == 200
    # a callback error aborts immediately (record.go:260-262)
    calls = []

    def cb(r, f, s):
        calls.append(f)
        return RuntimeError("stop") if len(calls) == 7 else None
    with pytest.raises(RuntimeError):
        W.iterate_record(W.load_wal(data), cb, 20, 20, ctx)
    assert len(calls) == 7


def test_iterate_hint_replay(ctx):
    data, payloads, offs = mixed_wal(4)
    ec, _, _, hint = O.hint_by_wal(data, 11, 40, BASE, 20, 20)
    assert ec == 0
    got = []
    W.iterate_hint(W.load_wal(hint, fid=11), got.append, 20, ctx)
    assert len(got) == len(payloads)
    ref = oracle_records(data)
    for i, h in enumerate(got):
        assert (h.fid, h.off, h.size) == (11, offs[i], len(payloads[i]))
        rr = ref.recs[i]
        hs = int(rr["hdr_size"])
        assert h.key == ref.payloads[i][hs:hs + int(rr["key_len"])]
    # a corrupted hint record mid-file: ErrCorruptedHintRecord after the rows before it
    w = O.Writer(BASE, BASE)
    for i in range(50):
        w.write(O.hint_encode(b"N" * 20, b"k%d" % i, 3, 40 + i, 100) if i != 30 else b"N" * 20 + b"\x05ab")
    got = []
    with pytest.raises(W.ErrCorruptedHintRecord):
        W.iterate_hint(W.load_wal(w.data(), fid=3), got.append, 20, ctx)
    assert len(got) == 30


def test_compact_one_wal_with_filter_callback(ctx):
    """compactOneWal with a doFilter callback (compaction.go:299-311): the filter is called in record order,
    the kept records' bytes equal the oracle's, and the filter is NOT called past the first row whose
    Record.Encode fails (the reference returns there)."""
    data, payloads, offs = mixed_wal(5)
    src = W.load_wal(data, fid=2)
    rng = random.Random(9)
    verdict = [rng.random() < 0.3 for _ in payloads]  # True = drop
    seen = []

    def flt(rec, fid, off):
        seen.append(off)
        assert fid == 2
        return verdict[len(seen) - 1]
    dst, hint = W.WalFile(7, BASE), W.WalFile(7, BASE)
    offs_out = W.compact_one_wal(dst, hint, src, flt, 20, 20, ctx)
    assert seen == offs
    keep = np.array([not v for v in verdict], dtype=np.uint8)
    rd, rh = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
    ec, _, nin, roffs = O.compact_append(rd, rh, 7, data, 40, BASE, BASE, 20, 20, keep)
    assert ec == 0 and bytes(dst.data) == rd.data() and bytes(hint.data) == rh.data()
    np.testing.assert_array_equal(offs_out[:nin], roffs[:nin])
    # an expire below the dst baseTime on a kept row: "invalid expire", and the filter stops there
    pl = [cases.rec(i, vlen=50) for i in range(40)]
    pl[25] = cases.rec(25, vlen=50, expire=BASE + 3)
    data2, offs2 = cases.wal_of(pl)
    seen.clear()
    calls = []

    def keep_all(rec, fid, off):
        calls.append(off)
        return False
    dst, hint = W.WalFile(8, BASE + 10), W.WalFile(8, BASE + 10)
    with pytest.raises(W.WalError, match="invalid expire"):
        W.compact_one_wal(dst, hint, W.load_wal(data2, fid=1), keep_all, 20, 20, ctx)
    assert calls == offs2[:26]
    rd, rh = O.Writer(BASE + 10, BASE + 10), O.Writer(BASE + 10, BASE + 10)
    ec, er, _, _ = O.compact_append(rd, rh, 8, data2, 40, BASE, BASE + 10, 20, 20, np.ones(40, dtype=np.uint8))
    assert ec == L.ENC_ERR_EXPIRE and er == 25
    assert bytes(dst.data) == rd.data() and bytes(hint.data) == rh.data()


def test_new_hint_by_wal_error_replay(ctx):
    data, _, _ = mixed_wal(6, bad_row=77)
    with pytest.raises(W.ErrInvalidData):
        W.new_hint_by_wal(W.load_wal(data, fid=3), 20, 20, ctx)
    ok, payloads, offs = mixed_wal(7)
    h = W.new_hint_by_wal(W.load_wal(ok, fid=3), 20, 20, ctx)
    ec, _, _, ref = O.hint_by_wal(ok, 3, 40, BASE, 20, 20)
    assert bytes(h.data) == ref


def test_encode_rec_off_capacity_and_zero_length_fulls(ctx):
    """a WAL of zero-length Full fragments (7-byte records, ~4681 per block): n_records is huge, every row
    is invalid data, so nothing is written; rec_off copies are bounded by rec_off_cap."""
    hdr = (0xA282EAD8).to_bytes(4, "little") + b"\x00\x00\x01"
    sb = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(sb, BASE, BASE)
    data = bytes(sb) + (hdr * 4681 + b"\0") * 3  # 4681 headers fill a block up to one pad byte
    res, wal, hb, offs = ctx.encode(data, L.ENC_COMPACT, 40, BASE, 9, 40, 40, 20, 20, np.ones(20000, np.uint8))
    assert res.err_class == L.ENC_ERR_SRC and res.err_record == 0 and res.n_in == 0
    assert wal == b"" and hb == b"" and offs.size == 0
    # direct call with a guarded rec_off buffer
    src = np.frombuffer(O.synth(1 << 40, 300, 1), dtype=np.uint8)
    p = L.EncodeParams(src.size, BASE, 9, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    keep = np.ones(300, dtype=np.uint8)
    wbuf = np.zeros(src.size * 2, dtype=np.uint8)
    hbuf = np.zeros(1 << 20, dtype=np.uint8)
    roff = np.full(400, 7, dtype=np.uint64)
    out = L.EncodeOut(wbuf.ctypes.data_as(L.u8p), wbuf.size, hbuf.ctypes.data_as(L.u8p), hbuf.size,
                      roff.ctypes.data_as(L.u64p), 100)
    r = L.EncodeResult()
    rc = L.lib.bcw_encode_segment(ctx.handle, src.ctypes.data_as(C.c_void_p), C.byref(p),
                                  keep.ctypes.data_as(C.c_void_p), keep.size, C.byref(out), C.byref(r))
    assert rc == L.E_CAPACITY and r.n_in == 300
    assert (roff == 7).all()  # nothing copied
    out.rec_off_cap = 400
    rc = L.lib.bcw_encode_segment(ctx.handle, src.ctypes.data_as(C.c_void_p), C.byref(p),
                                  keep.ctypes.data_as(C.c_void_p), keep.size, C.byref(out), C.byref(r))
    assert rc == 0 and r.err_class == 0 and r.n_written == 300
    assert (roff[300:] == 7).all() and (roff[:300] != 7).all()


def test_encode_async_generation_and_table_checks():
    """bcw_encode_segment_async refuses a decode result that is not the context's latest decode
    (BCW_ENC_ERR_STALE) and a source table smaller than the decode (BCW_ENC_ERR_TABLE)."""
    import _devmem as D
    from bitcaskdb_amd import Context
    c = Context(0)
    data = O.synth(1 << 40, 500, 3)
    src = D.upload(data)
    ec, _, _, hint = O.hint_by_wal(data, 3, 40, BASE, 20, 20)
    hsrc = D.upload(hint)
    tab, htab, small = D.DevTable(600), D.DevTable(600), D.DevTable(100)
    rsz = C.sizeof(L.DecodeResult)
    d_res, h_res = D.DevBuf(rsz), D.DevBuf(rsz)
    e_res = D.DevBuf(C.sizeof(L.EncodeResult))
    keep = D.DevBuf(600, fill=1)
    wout, hout, roff = D.DevBuf(len(data) * 2), D.DevBuf(1 << 20), D.DevBuf(600 * 8)
    dp = L.DecodeParams(len(data), BASE, 40, 20, 20, L.MODE_RECORD)
    hp = L.DecodeParams(len(hint), BASE, 40, 20, 0, L.MODE_HINT)
    ep = L.EncodeParams(len(data), BASE, 9, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    out = L.EncodeOut(C.cast(wout.vp(), L.u8p), wout.n, C.cast(hout.vp(), L.u8p), hout.n, C.cast(roff.vp(), L.u64p), 0)

    def dec(params, t, r, buf):
        assert L.lib.bcw_decode_segment_async(c.handle, buf.vp(), C.byref(params), C.byref(t.t), r.vp()) == 0

    def enc(t, r):
        assert L.lib.bcw_encode_segment_async(c.handle, src.vp(), C.byref(ep), C.byref(t.t), r.vp(), keep.vp(),
                                              C.byref(out), e_res.vp()) == 0
        c.sync()
        return L.EncodeResult.from_buffer_copy(bytes(e_res.download()))

    dec(dp, tab, d_res, src)
    dec(hp, htab, h_res, hsrc)  # replaces the context's fragment table
    r = enc(tab, d_res)
    assert r.err_class == L.ENC_ERR_STALE and r.wal_need == 0 and r.n_written == 0
    dec(dp, tab, d_res, src)
    r = enc(tab, d_res)
    assert r.err_class == 0 and r.n_written == 500
    rd, rh = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
    O.compact_append(rd, rh, 9, data, 40, BASE, BASE, 20, 20, np.ones(500, np.uint8))
    assert bytes(wout.download(r.wal_need)) == rd.data()[40:]
    dec(dp, small, d_res, src)
    r = enc(small, d_res)
    assert r.err_class == L.ENC_ERR_TABLE and r.n_written == 0 and r.wal_need == 0
    c.close()


def test_two_contexts_two_threads():
    """compaction, hint rebuild and recovery may overlap: two contexts driven from two
    threads at once (ctypes releases the GIL in the calls), every result checked against the oracle."""
    from bitcaskdb_amd import Context
    inputs = [O.synth(6 << 20, 0, 100 + k, value_mode=k % 2) for k in range(4)]
    refs = [O.decode(d, 40, BASE, 20, 20, want_bytes=False) for d in inputs]
    hrefs = [O.hint_by_wal(d, 5, 40, BASE, 20, 20)[3] for d in inputs]
    errors = []

    def worker(tid):
        try:
            c = Context(0)
            for it in range(6):
                k = (tid + it) % len(inputs)
                dec = c.decode(np.frombuffer(inputs[k], dtype=np.uint8), 40, BASE, 20, 20)
                if dec.n_records != len(refs[k].recs) or not np.array_equal(dec.table["foff"], refs[k].recs["foff"]):
                    errors.append(f"thread {tid} decode {k}")
                res, _, hb, _ = c.encode(inputs[k], L.ENC_HINT, 40, BASE, 5, 40, 40, 20, 20)
                if hb != hrefs[k][40:]:
                    errors.append(f"thread {tid} hint {k}")
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {tid}: {e!r}")
    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
