"""GPU parity of the batched point reads (bcw_read_records) against oc_read_record
(Wal.ReadRecord + WalParseRecord, pinned in test_oracle_read.py) and oc_record_parse (RecordFromBytes):
the reference's ReadRecord scenarios, every error branch, and seeded fuzz of (offset, size) requests
over valid, corrupted and mis-sized index values, with and without checksum verification."""
from __future__ import annotations

import random

import numpy as np
import pytest

import _oracle as O
import cases
from bitcaskdb_amd import _lib as L
from bitcaskdb_amd import wal as W

pytestmark = pytest.mark.gpu
BASE = cases.BASE
REC_FIELDS = ("expire", "key_len", "val_len", "meta_len", "hdr_size", "flags", "etag_off", "status")


def check(ctx, data, offs, sizes, verify=True, ns=20, etag=20):
    pays, st, tab = ctx.read_records(data, offs, sizes, BASE, ns, etag, verify)
    for i, (o, z) in enumerate(zip(offs, sizes)):
        ost, opay = O.read_record(data, o, z, verify)
        assert st[i] == ost, (i, o, z, st[i], ost)
        if ost == 0:
            assert pays[i] == opay, i
            r = O.record_parse(opay, BASE, ns, etag)
            for f in REC_FIELDS:
                assert int(tab[f][i]) == int(r[f]), (i, f, int(tab[f][i]), int(r[f]))
            assert int(tab["foff"][i]) == o + 7 and int(tab["size"][i]) == z
    return st


def test_reference_read_scenarios(ctx):
    """wal_test.go:17-237 shapes: small records, a 2-block record, 1000 x 5 KiB, block padding"""
    recs = [b"hello world", b"first record", bytes(i % 256 for i in range(65536)), bytes(32761),
            b"new block record"] + [bytes(i % 251 for i in range(5120))] * 1000
    data, offs = cases.wal_of(recs)
    for verify in (True, False):
        st = check(ctx, data, offs, [len(r) for r in recs], verify)
        assert (st == 0).all()


def test_read_records_payloads(ctx):
    """valid records of every shape (etag, expire, tombstone, meta, large values): Record fields"""
    data, p = cases.case_records_mixed()
    dec = O.decode(data, 40, BASE, 20, 20)
    offs = [int(f) - 7 for f in dec.recs["foff"]]
    sizes = [int(s) for s in dec.recs["size"]]
    st = check(ctx, data, offs, sizes)
    assert (st == 0).all()
    got = W.read_records(W.load_wal(data), offs, sizes)
    assert all(isinstance(x, W.Record) for x in got)


def test_read_error_branches(ctx):
    rec = bytes(range(200))
    data, offs = cases.wal_of([rec, rec, bytes(40000)])
    o = offs[0]
    bad = bytearray(data)
    bad[o + 2:o + 4] = b"\xff\xff"  # TestWal_CorruptedRead
    bad[offs[1] + 6] = 9            # unknown type
    reqs = [(o, 200), (o, 201), (o, 199), (o, 0), (len(data) - 10, 100), (offs[1], 200),
            (offs[2], 32768 - 40 - 7 + 3), (offs[2], 40000), (offs[2], 39999), (offs[2], 40001),
            (offs[2], 32768 - (offs[2] - 40) % 32768 - 7)]  # exactly the First fragment: incomplete
    seen = set()
    for verify in (True, False):
        seen |= set(check(ctx, bytes(bad), [a for a, _ in reqs], [b for _, b in reqs], verify).tolist())
    assert {L.RD_OK, L.RD_PANIC, L.RD_BEYOND, L.RD_SIZE, L.RD_CORRUPTED, L.RD_CRC, L.RD_TYPE,
            L.RD_INCOMPLETE} <= seen
    got = W.read_records(W.load_wal(bytes(bad)), [o, offs[1]], [200, 200])
    assert isinstance(got[0], W.ErrWalMismatchCRC) and isinstance(got[1], W.ErrWalUnknownRecordType)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_read_fuzz(ctx, seed):
    rng = random.Random(seed)
    payloads = [cases.rec(i, vlen=rng.choice([0, 5, 300, 5000, 32761 - 60, 40000, 70000])) for i in range(120)]
    data, offs = cases.wal_of(payloads)
    data = bytearray(data)
    for _ in range(6):  # scattered corruption
        data[rng.randrange(40, len(data))] ^= 1 << rng.randrange(8)
    data = bytes(data)
    ro, rs = [], []
    for _ in range(3000):
        k = rng.randrange(len(payloads))
        o, z = offs[k], len(payloads[k])
        m = rng.random()
        if m < 0.15:
            z += rng.choice([-1, 1, -7, 7, 32768])
            z = max(z, 0)
        elif m < 0.25:
            o = rng.randrange(0, len(data))
        elif m < 0.3:
            z = 0
        ro.append(o)
        rs.append(z)
    for verify in (True, False):
        st = check(ctx, data, ro, rs, verify)
        assert (st == 0).sum() > 1000


@pytest.mark.parametrize("vlen", [32761 - 60, 33000, 40000, 65400])
def test_read_crafted_long_full_fragment(ctx, vlen):
    """A crafted single Full fragment longer than a block's data area (u16 length up to 65535): WalParseRecord
    accepts it when it fits the span WalRecordSize computes. The verify path shifts lane chunks by up to the
    fragment length, so it needs the 2^15 shift operator (shifts of 32 KiB and more)."""
    payload = cases.rec(5, vlen=vlen)
    assert len(payload) < 65536
    sb = bytearray(40)
    sb[:] = O.Writer(BASE, BASE).data()[:40]
    hdr = O.compute_crc32(payload).to_bytes(4, "little") + len(payload).to_bytes(2, "little") + bytes([1])
    rs = O.wal_record_size(40, len(payload))
    data = bytes(sb) + hdr + payload
    data += bytes(40 + rs - len(data) + 16)
    bad = bytearray(data)
    bad[40 + 7 + len(payload) - 3] ^= 0x10  # flips a byte near the end: only the high lanes' chunks change
    for img in (data, bytes(bad)):
        st = check(ctx, img, [40, 40, 40], [len(payload), len(payload) - 1, len(payload) + 1], verify=True)
        assert st[0] == (L.RD_OK if img is data else L.RD_CRC), st
