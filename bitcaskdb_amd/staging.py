"""Host I/O staging between WAL files and device memory, over bcw_stage (bcw_io.cpp).

The reference reads a segment 32 KiB at a time with PreadFull (utils.go:32-48, wal_iterator.go:55) and
writes the rewritten WAL through a buffer flushed every >= 1 MiB (WalRewriter wal_rewriter.go:37-49 ->
Wal.Flush wal.go:451-465). Here whole segments move between files and HBM through pinned slices: reader
threads pread while earlier slices cross PCIe, and device output is copied back and pwritten slice by
slice. Device buffers are plain device pointers (ints), e.g. torch tensors' data_ptr().
"""
from __future__ import annotations

import ctypes as C
import os

from . import _lib as L
from .wal import Context, default_context


class Stage:
    """bcw_stage: `nslices` pinned host buffers of `slice_bytes` bound to a context."""

    def __init__(self, ctx: Context | None = None, slice_bytes: int = 8 << 20, nslices: int = 8):
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        rc = L.lib.bcw_stage_create(self.ctx.handle, slice_bytes, nslices, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"bcw_stage_create: {L.lib.bcw_strerror(rc).decode()}")
        self._h = h

    def close(self):
        if self._h:
            L.lib.bcw_stage_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read(self, fd: int, file_off: int, length: int, d_dst: int, stream: int | None = None, threads: int = 4):
        """length bytes of fd at file_off into device memory at d_dst (copies queued on `stream`)."""
        rc = L.lib.bcw_stage_read(self._h, fd, file_off, length, C.c_void_p(d_dst), C.c_void_p(stream or 0), threads)
        if rc != 0:
            raise OSError(f"bcw_stage_read: {L.lib.bcw_strerror(rc).decode()}")

    def write(self, fd: int, file_off: int, d_src: int, length: int, stream: int | None = None, threads: int = 4):
        """length bytes of device memory at d_src into fd at file_off (after the work queued on `stream`)."""
        rc = L.lib.bcw_stage_write(self._h, fd, file_off, C.c_void_p(d_src), length, C.c_void_p(stream or 0), threads)
        if rc != 0:
            raise OSError(f"bcw_stage_write: {L.lib.bcw_strerror(rc).decode()}")

    def read_file(self, path: str, d_dst: int, stream: int | None = None, threads: int = 4) -> int:
        """the whole file into d_dst; returns its size"""
        fd = os.open(path, os.O_RDONLY)
        try:
            n = os.fstat(fd).st_size
            self.read(fd, 0, n, d_dst, stream, threads)
            return n
        finally:
            os.close(fd)

    def append_file(self, path: str, d_src: int, length: int, stream: int | None = None, threads: int = 4):
        """append length device bytes to a file (Wal.Flush of the rewriter's buffered output)"""
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            self.write(fd, os.fstat(fd).st_size, d_src, length, stream, threads)
        finally:
            os.close(fd)


def peer_enable(device_a: int, device_b: int):
    """bcw_peer_enable: each of the two devices may map the other's memory (xGMI peer access)"""
    rc = L.lib.bcw_peer_enable(device_a, device_b)
    if rc != 0:
        raise OSError(f"bcw_peer_enable({device_a}, {device_b}): {L.lib.bcw_strerror(rc).decode()}")


def peer_copy(ctx: Context, d_dst: int, d_src: int, src_device: int, length: int, stream: int | None = None):
    """bcw_stage_peer: length bytes of a segment resident on src_device -> d_dst on the context's device, device to
    device (over xGMI between linked GPUs), queued on the context's stream (or `stream`)"""
    rc = L.lib.bcw_stage_peer(ctx.handle, C.c_void_p(d_dst), C.c_void_p(d_src), src_device, length,
                              C.c_void_p(stream) if stream else None)
    if rc != 0:
        raise OSError(f"bcw_stage_peer: {L.lib.bcw_strerror(rc).decode()}")

