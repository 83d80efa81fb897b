"""GPU encode parity: compaction re-encode (compactOneWal, compaction.go:294-327) and hint rebuild
(NewHintByWal, hint.go:123-161) on the MI355X against the CPU oracle, bit-exact on the appended WAL and
hint bytes, the offsets WriteRecord returns and the error outcome. Everything goes through the C-ABI
(bcw_encode_segment)."""
from __future__ import annotations

import random

import numpy as np
import pytest

import _oracle as O
import cases
from bitcaskdb_amd import _lib as L

pytestmark = pytest.mark.gpu
BASE = cases.BASE
U64MAX = np.iinfo(np.uint64).max


def make_src(payloads, base=BASE):
    data, _ = cases.wal_of(payloads, base)
    return data


def rec_of(rng, i, ns=20, etag_size=20, vlen=None, klen=None, kinds=True):
    key = bytes(rng.getrandbits(8) for _ in range(klen if klen is not None else rng.randrange(0, 40)))
    v = vlen if vlen is not None else rng.choice([0, 1, 13, 200, 4096, rng.randrange(0, 40000)])
    val = bytes((i * 31 + k) & 0xff for k in range(v))
    etag = b""
    expire = 0
    tomb = False
    meta = b""
    if kinds:
        if rng.random() < 0.4:
            etag = bytes(rng.getrandbits(8) for _ in range(etag_size))
        if rng.random() < 0.4:
            expire = BASE + rng.choice([0, 1, 127, 128, 100000, 1 << 30])
        tomb = rng.random() < 0.2
        r = rng.random()
        if r < 0.1:
            meta = b"\x81\xa3foo\xa3bar"
        elif r < 0.15:
            meta = rng.choice([b"\x80", b"\xc0", b"\x81\xa0\xa0", b"\x82\xa0\xa0\xa0\xc0"])  # AppMetaSize 0
    nsb = bytes((65 + k) for k in range(ns))
    return O.record_encode(nsb, key, val, etag, expire, tomb, meta, BASE)


def prefill(rng, w, nbytes):
    while w.size() < nbytes:
        w.write(bytes(rng.getrandbits(8) for _ in range(rng.randrange(5, 3000))))


def run_compact(ctx, src, keep, ns=20, etag=20, dst_base=BASE, fid=9, pre_wal=0, pre_hint=0, seed=0):
    rng = random.Random(seed)
    dst, hint = O.Writer(dst_base, dst_base), O.Writer(dst_base, dst_base)
    prefill(rng, dst, pre_wal)
    prefill(rng, hint, pre_hint)
    wal_pos, hint_pos = dst.size(), hint.size()
    ec, er, nin, offs = O.compact_append(dst, hint, fid, src, 40, BASE, dst_base, ns, etag, keep)
    res, wal, hb, goffs = ctx.encode(src, L.ENC_COMPACT, 40, dst_base, fid, wal_pos, hint_pos, ns, etag, keep)
    assert res.err_class == ec, (res.err_class, ec, res.err_record, er)
    if ec in (L.ENC_ERR_EXPIRE, L.ENC_ERR_PANIC) or (ec == L.ENC_ERR_SRC and er >= 0):
        assert res.err_record == er
    assert res.n_in == nin
    ref_wal, ref_hint = dst.data()[wal_pos:], hint.data()[hint_pos:]
    assert res.wal_end == dst.size() and res.hint_end == hint.size()
    assert len(wal) == len(ref_wal)
    if wal != ref_wal:
        d = next(i for i in range(len(wal)) if wal[i] != ref_wal[i])
        raise AssertionError(f"dst WAL differs at file offset {wal_pos + d} (appended byte {d} of {len(wal)})")
    if hb != ref_hint:
        d = next((i for i in range(min(len(hb), len(ref_hint))) if hb[i] != ref_hint[i]), min(len(hb), len(ref_hint)))
        raise AssertionError(f"hint WAL differs at appended byte {d} ({len(hb)} vs {len(ref_hint)})")
    np.testing.assert_array_equal(goffs[:nin], offs[:nin])
    return res


@pytest.mark.parametrize("seed", range(6))
def test_compact_mixed(ctx, seed):
    rng = random.Random(seed)
    payloads = [rec_of(rng, i) for i in range(rng.randrange(50, 400))]
    src = make_src(payloads)
    keep = np.array([rng.random() < 0.7 for _ in payloads], dtype=np.uint8)
    run_compact(ctx, src, keep, pre_wal=rng.choice([0, 40, 1000, 32768 - 3, 32768 + 33, 100000]),
                pre_hint=rng.choice([0, 500, 32760]), seed=seed, dst_base=BASE - rng.choice([0, 0, 5, 1000]))


@pytest.mark.parametrize("target", [32761, 32761 - 7, 16377, (32768 - 14) // 2, 32768 - 9, 4222, 10919, 65536])
def test_compact_layout_events(ctx, target):
    """payload sizes that make blocks end exactly at record headers (exact fills, pads, zero-length Firsts)."""
    rng = random.Random(target)
    ns = 20
    payloads = []
    for i in range(60):
        t = target + rng.choice([0, 0, 0, -1, 1, -7, 7, -6])
        base = rec_of(rng, i, ns=ns, vlen=0, klen=8, kinds=False)
        payloads.append(rec_of(random.Random(i), i, ns=ns, vlen=max(0, t - len(base) - 2), klen=8, kinds=False))
    src = make_src(payloads)
    keep = np.ones(len(payloads), dtype=np.uint8)
    for pre in (0, 7, 32768 - 47, 32768 - 60):
        run_compact(ctx, src, keep, pre_wal=pre, pre_hint=pre, seed=pre)


def test_compact_tiny_records(ctx):
    """NsSize 0, empty keys/values: 5-byte payloads, ~2700 fragments per output block (one wave per
    12-byte record, every unit an edge unit)."""
    rng = random.Random(3)
    payloads = [O.record_encode(b"", b"", b"", b"", 0, False, b"", BASE) for _ in range(20000)]
    payloads += [rec_of(rng, i, ns=0, vlen=rng.randrange(0, 30), klen=rng.randrange(0, 4)) for i in range(5000)]
    src = make_src(payloads)
    keep = np.array([rng.random() < 0.9 for _ in payloads], dtype=np.uint8)
    run_compact(ctx, src, keep, ns=0, etag=4, pre_wal=123, pre_hint=0)


def test_compact_large_records(ctx):
    rng = random.Random(4)
    payloads = [rec_of(rng, i, vlen=rng.choice([70000, 200000, 32761, 5]), klen=100) for i in range(24)]
    src = make_src(payloads)
    keep = np.array([i % 3 != 1 for i in range(len(payloads))], dtype=np.uint8)
    run_compact(ctx, src, keep, pre_wal=5000, pre_hint=77)


@pytest.mark.parametrize("ns", [60, 100, 150])
def test_compact_large_namespace(ctx, ns):
    """NsSize large enough that a record's (or hint's) re-encoded header bytes exceed the writer's
    96-byte literal descriptor: those records take the bytewise general path."""
    rng = random.Random(ns)
    payloads = [rec_of(rng, i, ns=ns) for i in range(300)]
    src = make_src(payloads)
    keep = np.array([rng.random() < 0.8 for _ in payloads], dtype=np.uint8)
    run_compact(ctx, src, keep, ns=ns, pre_wal=32768 - 50, pre_hint=100, seed=ns)
    run_hint(ctx, src, ns=ns)


def test_compact_config_shape(ctx):
    """config E shape (ns 20, key 100, value 4096, everything kept) at 20k records."""
    src = O.synth(1 << 40, 20000, 42)
    keep = np.ones(20000, dtype=np.uint8)
    res = run_compact(ctx, src, keep)
    assert res.n_written == 20000


def test_compact_errors(ctx):
    rng = random.Random(7)
    payloads = [rec_of(rng, i, kinds=False) for i in range(100)]
    # invalid expire: record 40 expires before the dst baseTime
    payloads[40] = O.record_encode(b"A" * 20, b"k", b"v", b"", BASE + 10, False, b"", BASE)
    src = make_src(payloads)
    keep = np.ones(len(payloads), dtype=np.uint8)
    r = run_compact(ctx, src, keep, dst_base=BASE + 11)
    assert r.err_class == L.ENC_ERR_EXPIRE and r.err_record == 40
    # the same record dropped by the filter: no error
    keep2 = keep.copy()
    keep2[40] = 0
    r = run_compact(ctx, src, keep2, dst_base=BASE + 11)
    assert r.err_class == L.ENC_ERR_NONE
    # Record.Encode panic: expire delta >= 2^35 against the dst baseTime
    payloads[60] = O.record_encode(b"A" * 20, b"k", b"v", b"", BASE + (1 << 35) - 1, False, b"", BASE)
    src = make_src(payloads)
    r = run_compact(ctx, src, keep2, dst_base=BASE - 1)
    assert r.err_class == L.ENC_ERR_PANIC and r.err_record == 60
    # source corruption: the iteration stops at the CRC error, earlier records are written
    bad = bytearray(make_src([rec_of(rng, i, kinds=False) for i in range(200)]))
    bad[len(bad) // 2] ^= 0x10
    r = run_compact(ctx, bytes(bad), np.ones(200, dtype=np.uint8))
    assert r.err_class == L.ENC_ERR_SRC and r.src_err_class == L.ERR_CRC
    # an invalid record (RecordFromBytes error) mid-file
    payloads = [rec_of(rng, i, kinds=False) for i in range(50)]
    payloads[20] = b"\x05garbage-bytes"
    r = run_compact(ctx, make_src(payloads), np.ones(50, dtype=np.uint8))
    assert r.err_class == L.ENC_ERR_SRC and r.err_record == 20


def run_hint(ctx, src, ns=20, etag=20, fid=5):
    ec, er, nin, ref = O.hint_by_wal(src, fid, 40, BASE, ns, etag)
    res, _, hb, _ = ctx.encode(src, L.ENC_HINT, 40, BASE, fid, 40, 40, ns, etag)
    assert res.err_class == ec and res.n_in == nin
    assert hb == ref[40:], "hint WAL bytes differ"
    return res


def test_hint_by_wal(ctx):
    rng = random.Random(11)
    run_hint(ctx, make_src([rec_of(rng, i) for i in range(500)]))
    run_hint(ctx, O.synth(1 << 40, 3000, 1, value_mode=1))


def test_hint_by_wal_zero_length_first(ctx):
    """a zero-length First (7 bytes left in a block) shifts the iterator offset the hint carries
    (SURVEY.md 8.2 quirk 1)."""
    ns = 20
    first = rec_of(random.Random(0), 0, ns=ns, vlen=0, klen=8, kinds=False)
    # first record fills the block up to exactly 7 bytes before its end
    target = 32768 - 7 - 7
    filler = rec_of(random.Random(0), 0, ns=ns, vlen=target - len(first) - 2, klen=8, kinds=False)
    filler = filler if len(filler) == target else None
    assert filler is not None
    payloads = [filler] + [rec_of(random.Random(i), i, ns=ns, vlen=300, klen=8, kinds=False) for i in range(1, 40)]
    src = make_src(payloads)
    d = O.decode(src, 40, BASE, ns, 20)
    assert d.recs["foff"][1] - 7 == 40 + 32768  # the shifted iterator offset
    run_hint(ctx, src, ns=ns)
    run_compact(ctx, src, np.ones(len(payloads), dtype=np.uint8))


def test_roundtrip_decode_of_encoded(ctx):
    """the compacted WAL decodes (GPU) to the kept records with the returned offsets."""
    rng = random.Random(21)
    payloads = [rec_of(rng, i) for i in range(300)]
    src = make_src(payloads)
    keep = np.array([rng.random() < 0.5 for _ in payloads], dtype=np.uint8)
    res, wal, hb, offs = ctx.encode(src, L.ENC_COMPACT, 40, BASE, 3, 40, 40, 20, 20, keep)
    sb = bytearray(40)
    import ctypes as C
    buf = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(buf, BASE, BASE)
    image = bytes(buf) + wal
    dec = ctx.decode(np.frombuffer(image, dtype=np.uint8), 40, BASE, 20, 20)
    assert dec.result.err_class == 0
    assert dec.n_records == int(keep.sum())
    written = offs[offs != U64MAX]
    np.testing.assert_array_equal(dec.table["foff"] - 7, written)
    hdec = ctx.decode(np.frombuffer(bytes(buf) + hb, dtype=np.uint8), 40, BASE, 20, 0, L.MODE_HINT)
    assert hdec.n_records == int(keep.sum())
    np.testing.assert_array_equal(hdec.table["aux0"], written)
    del sb


@pytest.mark.parametrize("wal_pos,hint_pos", [((1 << 35) + 12345, (1 << 32) + 777),
                                              ((1 << 32) - 3_000_000, (1 << 28) - 100_000),
                                              ((1 << 40) + 32768 - 3, (1 << 33) + 7)])
def test_compact_config_e_large_offsets(ctx, wal_pos, hint_pos):
    """config E's regime (a 42.3 GB dst WAL): appends of config-E-shape records (NsSize 20, 100 B keys, 4 KiB values)
    at dst positions past 2^32 and 2^35 (WriteRecord offsets above 32 bits, hint `off` varints of 5 and 6 bytes,
    hint.go:32-48) and crossing 2^32 inside the batch, hint positions past 2^28 / 2^32 -- against oc_compact_append on
    writers opened at those positions (wal.go:482-516: the layout depends on the position only through its block
    phase, the returned offsets and hint fields on the position itself)"""
    src = np.frombuffer(O.synth(8 << 20, 0, 77, 20, 100, 4096, 0, BASE), dtype=np.uint8)
    n_rec = len(O.decode(src, 40, BASE, 20, 20, want_bytes=False).recs)
    keep = np.ones(n_rec, dtype=np.uint8)
    keep[::97] = 0  # a few dropped rows: the dense layout has gaps in the source
    dst, hint = O.Writer(BASE, BASE, at=wal_pos), O.Writer(BASE, BASE, at=hint_pos)
    ec, er, nin, offs = O.compact_append(dst, hint, 5, src, 40, BASE, BASE, 20, 20, keep)
    assert ec == 0 and nin == n_rec
    assert int(offs[keep.astype(bool)].max()) > wal_pos  # the offsets really are that large
    res, wal, hb, goffs = ctx.encode(src, L.ENC_COMPACT, 40, BASE, 5, wal_pos, hint_pos, 20, 20, keep)
    assert res.err_class == 0 and res.n_in == nin
    assert res.wal_end == dst.size() and res.hint_end == hint.size()
    assert wal == dst.data(), "dst WAL bytes differ"
    assert hb == hint.data(), "hint WAL bytes differ"
    np.testing.assert_array_equal(goffs[:nin], offs[:nin])
