"""GPU tests of the host I/O staging (bcw_stage): file -> pinned slices -> HBM and back,
byte-exact, and an end-to-end compaction file -> device decode -> encode -> file equal to the oracle's."""
from __future__ import annotations

import os

import numpy as np
import pytest

import _devmem as D
import _oracle as O
import cases
from bitcaskdb_amd import _lib as L
from bitcaskdb_amd import Stage

pytestmark = pytest.mark.gpu
BASE = cases.BASE


@pytest.mark.parametrize("size,slice_,threads", [(1, 4096, 1), (4096 * 3 + 17, 4096, 3), (20 << 20, 1 << 20, 4),
                                                  ((64 << 20) + 12345, 8 << 20, 8)])
def test_stage_roundtrip(ctx, tmp_path, size, slice_, threads):
    rng = np.random.default_rng(size)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    src = tmp_path / "src.bin"
    src.write_bytes(data.tobytes())
    st = Stage(ctx, slice_, 4)
    buf = D.DevBuf(size + 100)
    assert st.read_file(str(src), buf.ptr + 3, threads=threads) == size
    ctx.sync()
    assert bytes(buf.download(size, 3)) == data.tobytes()
    dst = tmp_path / "dst.bin"
    dst.write_bytes(b"HEAD")
    st.append_file(str(dst), buf.ptr + 3, size, threads=threads)
    assert dst.read_bytes() == b"HEAD" + data.tobytes()
    # a short file is an I/O error, as a truncated pread
    with pytest.raises(OSError):
        fd = os.open(str(src), os.O_RDONLY)
        try:
            st.read(fd, 0, size + 1, buf.ptr)
        finally:
            os.close(fd)
    st.close()


@pytest.mark.parametrize("size", [4096, (9 << 20) + 4096 * 3 + 123])
def test_stage_read_odirect(ctx, tmp_path, size):
    """an O_DIRECT descriptor (reads past the page cache): whole-4-KiB requests, the short tail at end of file;
    unaligned offsets are refused. Skipped where the filesystem refuses O_DIRECT (tmpfs)."""
    rng = np.random.default_rng(size)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    src = tmp_path / "src.bin"
    src.write_bytes(data.tobytes())
    try:
        fd = os.open(str(src), os.O_RDONLY | os.O_DIRECT)
    except OSError as e:
        pytest.skip(f"O_DIRECT refused here: {e.strerror}")
    st = Stage(ctx, 1 << 20, 4)
    buf = D.DevBuf(size + 64)
    try:
        st.read(fd, 0, size, buf.ptr, threads=3)
        ctx.sync()
        assert bytes(buf.download(size)) == data.tobytes()
        with pytest.raises(OSError):
            st.read(fd, 100, 4096, buf.ptr)  # not 4 KiB-aligned
    finally:
        os.close(fd)
        st.close()


def test_file_to_file_compaction(ctx, tmp_path):
    """a data WAL on disk -> staged into HBM -> decode -> re-encode (all kept) and hint rebuild on the device
    -> staged back to the dst WAL / hint files: the files equal the oracle's."""
    import ctypes as C
    data = O.synth(24 << 20, 0, 9, value_mode=1)
    src = tmp_path / "1.wal"
    src.write_bytes(data)
    st = Stage(ctx, 1 << 20, 4)
    d_src = D.DevBuf(len(data))
    st.read_file(str(src), d_src.ptr)
    n_rows = len(data) // 64 + 64
    tab = D.DevTable(n_rows)
    d_res = D.DevBuf(C.sizeof(L.DecodeResult))
    dp = L.DecodeParams(len(data), BASE, 40, 20, 20, L.MODE_RECORD)
    assert L.lib.bcw_decode_segment_async(ctx.handle, d_src.vp(), C.byref(dp), C.byref(tab.t), d_res.vp()) == 0
    keep = D.DevBuf(n_rows, fill=1)
    wout, hout = D.DevBuf(len(data) + (1 << 20)), D.DevBuf(len(data) // 8 + (1 << 20))
    e_res = D.DevBuf(C.sizeof(L.EncodeResult))
    ep = L.EncodeParams(len(data), BASE, 2, 40, 40, 40, L.ENC_COMPACT, 20, 20)
    out = L.EncodeOut(C.cast(wout.vp(), L.u8p), wout.n, C.cast(hout.vp(), L.u8p), hout.n, None, 0)
    assert L.lib.bcw_encode_segment_async(ctx.handle, d_src.vp(), C.byref(ep), C.byref(tab.t), d_res.vp(), keep.vp(),
                                          C.byref(out), e_res.vp()) == 0
    ctx.sync()
    r = L.EncodeResult.from_buffer_copy(bytes(e_res.download()))
    assert r.err_class == 0 and r.fits
    sb = (C.c_uint8 * 40)()
    L.lib.bcw_write_super_block(sb, BASE, BASE)
    for name in ("2.merge", "2.tmp"):
        (tmp_path / name).write_bytes(bytes(sb))
    st.append_file(str(tmp_path / "2.merge"), wout.ptr, r.wal_need)
    st.append_file(str(tmp_path / "2.tmp"), hout.ptr, r.hint_need)
    rd, rh = O.Writer(BASE, BASE), O.Writer(BASE, BASE)
    dec = O.decode(data, 40, BASE, 20, 20, want_bytes=False)
    ec, _, nin, _ = O.compact_append(rd, rh, 2, data, 40, BASE, BASE, 20, 20, np.ones(len(dec.recs), np.uint8))
    assert ec == 0
    assert (tmp_path / "2.merge").read_bytes() == rd.data()
    assert (tmp_path / "2.tmp").read_bytes() == rh.data()


def test_peer_copy_then_decode(ctx):
    """bcw_stage_peer: a segment resident in another buffer of the GPU (the box has one device: the same-device
    branch; between two devices it is hipMemcpyPeerAsync over xGMI) copied device to device on the context's
    stream, then decoded: every column equals the oracle's. bcw_peer_enable of a device with itself is a no-op;
    out-of-range devices are refused."""
    import ctypes as C
    from bitcaskdb_amd.staging import peer_copy, peer_enable
    data = O.synth(8 << 20, 0, 77, value_mode=1)
    src = D.DevBuf(len(data))
    src.upload(np.frombuffer(data, np.uint8))
    dst = D.DevBuf(len(data) + 64)
    peer_enable(0, 0)
    with pytest.raises(OSError):
        peer_enable(0, 1 << 20)
    peer_copy(ctx, dst.ptr + 16, src.ptr, 0, len(data))
    ctx.sync()
    assert bytes(dst.download(len(data), 16)) == data
    n_rows = len(data) // 64 + 64
    tab = D.DevTable(n_rows)
    d_res = D.DevBuf(C.sizeof(L.DecodeResult))
    dp = L.DecodeParams(len(data), BASE, 40, 20, 20, L.MODE_RECORD)
    assert L.lib.bcw_decode_segment_async(ctx.handle, C.c_void_p(dst.ptr + 16), C.byref(dp), C.byref(tab.t),
                                          d_res.vp()) == 0
    ctx.sync()
    r = L.DecodeResult.from_buffer_copy(bytes(d_res.download()))
    ref = O.decode(data, 40, BASE, 20, 20, want_bytes=False)
    assert r.err_class == ref.err_class == 0 and r.n_records == len(ref.recs)
    np.testing.assert_array_equal(tab.column("foff", r.n_records), ref.recs["foff"])
    np.testing.assert_array_equal(tab.column("size", r.n_records), ref.recs["size"])
