"""The point-read oracle (oc_read_record: Wal.ReadRecord wal.go:556-573 + WalParseRecord wal.go:121-173)
pinned by the reference's own ReadRecord tests (wal_test.go:17-237, restated over the oracle writer)."""
from __future__ import annotations

import _oracle as O
import cases

BLOCK, HDR = 32768, 7


def test_basic_and_multiple():
    """TestWal_BasicOperations / TestWal_MultipleRecords (wal_test.go:17-70), verify on and off"""
    recs = [b"hello world", b"first record", b"second record", b"third record"]
    data, offs = cases.wal_of(recs)
    for r, o in zip(recs, offs):
        assert O.read_record(data, o, len(r), True) == (0, r)
        assert O.read_record(data, o, len(r), False) == (0, r)


def test_large_records():
    """TestWal_LargeRecord / LargeRecord2 (wal_test.go:73-115): 2 blocks of data; 1000 x 5 KiB"""
    big = bytes(i % 256 for i in range(BLOCK * 2))
    data, offs = cases.wal_of([big])
    assert O.read_record(data, offs[0], len(big)) == (0, big)
    five = bytes(i % 251 for i in range(5 * 1024))
    data, offs = cases.wal_of([five] * 1000)
    for o in offs:
        assert O.read_record(data, o, len(five)) == (0, five)


def test_corrupted_read():
    """TestWal_CorruptedRead (wal_test.go:118-155): 0xFFFF over bytes 2-3 of the record -> an error"""
    rec = b"valid record"
    data, offs = cases.wal_of([rec])
    bad = bytearray(data)
    bad[offs[0] + 2:offs[0] + 4] = b"\xff\xff"
    st, _ = O.read_record(bytes(bad), offs[0], len(rec), True)
    assert st == 3  # ErrWalMismatchCRC
    assert O.read_record(bytes(bad), offs[0], len(rec), False) == (0, rec)  # not verified: the data is intact


def test_block_padding():
    """TestWal_BlockPadding (wal_test.go:158-190)"""
    a, b = bytes(BLOCK - HDR), b"new block record"
    data, offs = cases.wal_of([a, b])
    assert O.read_record(data, offs[0], len(a)) == (0, a)
    assert O.read_record(data, offs[1], len(b)) == (0, b)


def test_error_classes():
    """each WalParseRecord / ReadRecord failure branch"""
    rec = bytes(range(200))
    data, offs = cases.wal_of([rec, rec])
    o = offs[0]
    assert O.read_record(data, o, len(rec) + 1)[0] == 4      # the Full fragment ends short: size mismatch
    assert O.read_record(data, o, len(rec) - 1)[0] == 2      # the Full fragment is longer than the buffer
    assert O.read_record(data, o, 0)[0] == 7                 # empty buffer: the header slice panics
    assert O.read_record(data, len(data) - 10, 100)[0] == 1  # read beyond file size
    bad = bytearray(data)
    bad[o + 6] = 9
    assert O.read_record(bytes(bad), o, len(rec), False)[0] == 5  # unknown type
    big = bytes(40000)
    data, offs = cases.wal_of([big])
    # a First fragment, then the buffer (sized for 100 bytes) ends: incomplete / corrupted
    st, _ = O.read_record(data, offs[0], 32768 - 40 - 7 + 3)
    assert st in (2, 6)
    assert O.read_record(data, offs[0], 40000) == (0, big)
    first = 32768 - (offs[0] - 40) % 32768 - 7
    assert O.read_record(data, offs[0], first)[0] == 6  # the buffer ends after the First fragment
