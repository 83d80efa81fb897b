"""CPU tests of the C-ABI library: it loads, exports every symbol include/bcw.h declares, and its
host-side helpers (no device work) agree with the oracle."""
from __future__ import annotations

import ctypes as C
import random
import struct

import numpy as np
import pytest

import _oracle as O
from bitcaskdb_amd import _lib as L
from bitcaskdb_amd import compute_crc32, load_wal
from bitcaskdb_amd import wal as W


def test_library_exports_every_header_symbol():
    syms = L.header_symbols()
    assert len(syms) >= 15
    for name in syms:
        assert hasattr(L.lib, name), f"libbcw.so does not export {name}"
    assert L.lib.bcw_abi_version() == 2
    assert L.lib.bcw_strerror(-4) == b"output capacity too small"


def test_crc_host_helper():
    assert compute_crc32(b"123456789") == 0xC78AB0E5
    assert compute_crc32(b"") == 0xA282EAD8
    rng = random.Random(3)
    for n in (1, 5, 64, 1000, 4097):
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert compute_crc32(b) == O.compute_crc32(b)


def test_super_block_roundtrip_and_errors():
    out = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(out, 123, 456)
    ref = np.zeros(40, dtype=np.uint8)
    O.lib.oc_super_encode(ref.ctypes.data_as(C.c_void_p), 123, 456)
    assert bytes(out) == bytes(ref)
    w = load_wal(bytes(out) + b"", fid=3)
    assert (w.start_off, w.base_time, w.create_time, w.fid) == (40, 456, 123, 3)
    bad = bytearray(out)
    bad[0] ^= 1
    with pytest.raises(W.ErrWalMismatchCRC):
        load_wal(bytes(bad))
    with pytest.raises(W.ErrShortFile):
        load_wal(bytes(out)[:39])
    # a valid CRC over a wrong magic / block size: checked in that order (wal.go:369-385)
    for field, exc in ((0, W.ErrWalMismatchMagic), (8, W.ErrWalMismatchBlockSize)):
        b = bytearray(out)
        b[field] ^= 0x10
        b[36:40] = struct.pack("<I", O.compute_crc32(bytes(b[:36])))
        with pytest.raises(exc):
            load_wal(bytes(b))


@pytest.mark.parametrize("cfg", [(1 << 20, 0, 0x5EED, 0), (3 << 20, 0, 42, 1), (0, 5, 9, 0), (2 << 20, 77, 1, 0)])
def test_product_writer_matches_oracle(cfg):
    target, maxrec, seed, mode = cfg
    target = target or (1 << 30)
    n, r = C.c_uint64(), C.c_uint64()
    assert L.lib.bcw_synth_segment(target, maxrec, seed, 20, 100, 4096, mode, 1_700_000_000, None, 0, C.byref(n),
                                   C.byref(r)) == 0
    buf = np.zeros(n.value, dtype=np.uint8)
    assert L.lib.bcw_synth_segment(target, maxrec, seed, 20, 100, 4096, mode, 1_700_000_000,
                                   buf.ctypes.data_as(C.c_void_p), buf.size, C.byref(n), C.byref(r)) == 0
    assert bytes(buf) == O.synth(target, maxrec, seed, value_mode=mode)


def test_max_fragments():
    assert L.lib.bcw_max_fragments(40, 40) == 0
    assert L.lib.bcw_max_fragments(47, 40) == 2
    assert L.lib.bcw_max_fragments(40 + 32768, 40) == 32768 // 7 + 1


def test_wal_record_size_and_block_range():
    """WalRecordSize / WalBlockIndexRange (wal.go:61-97) through the C-ABI against the oracle, and against
    the physical span the writer (wal.go:490-553) actually gives each record."""
    rng = random.Random(5)
    cases = [(40, 0), (40, 1), (40, 32761), (40, 32762), (32768 + 40 - 7, 10), (32768 + 40 - 6, 10),
             (32768 + 40 - 8, 1), (100, 200000), (2**40 + 40, 70000)]
    cases += [(40 + rng.randrange(0, 1 << 20), rng.choice([0, 1, 5, 4222, 32761, rng.randrange(0, 300000)]))
              for _ in range(300)]
    for off, size in cases:
        assert L.lib.bcw_wal_record_size(off, size) == O.wal_record_size(off, size), (off, size)
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        L.lib.bcw_wal_block_index_range(off, size, C.byref(a), C.byref(b), C.byref(c))
        assert (a.value, b.value, c.value) == O.wal_block_index_range(off, size), (off, size)
    # the footprint of every record the writer appends = the bytes from its offset to the next record's
    # first header or the padding before it (WalRecordSize counts no padding at the record start)
    w = O.Writer(1, 1)
    offs, sizes = [], []
    for i in range(400):
        n = rng.choice([5, 4222, 32761 - 7, 32761, 32754, rng.randrange(5, 70000)])
        offs.append(w.write(bytes(n)))
        sizes.append(n)
    end = w.size()
    for i, (off, n) in enumerate(zip(offs, sizes)):
        rs = int(L.lib.bcw_wal_record_size(off, n))
        nxt = offs[i + 1] if i + 1 < len(offs) else end
        pad = (32768 - (off + rs - 40) % 32768) if (off + rs - 40) % 32768 > 32768 - 7 else 0
        assert off + rs == nxt or off + rs + pad == nxt, (i, off, n, rs, nxt)


def test_reserve_fragments_rejects_oversize():
    # no device needed: the call only records a sizing hint (ctx NULL is refused)
    assert L.lib.bcw_ctx_reserve_fragments(None, 10) == -1


def test_host_murmur3_matches_oracle():
    from bitcaskdb_amd import murmur3_sum64
    rng = random.Random(8)
    for s in [b"", b"hello", b"hello, world", b"The quick brown fox jumps over the lazy dog."]:
        assert murmur3_sum64(s) == O.murmur3_sum64(s)
    assert murmur3_sum64(b"hello") == 0xcbd8a7b341bd9b02
    for n in range(0, 140):
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert murmur3_sum64(b) == O.murmur3_sum64(b)
