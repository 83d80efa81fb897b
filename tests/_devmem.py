"""Device buffers for the async C-ABI tests through the HIP runtime libbcw.so itself links
(libamdhip64.so.7): hipMalloc / hipMemcpy / hipFree via ctypes. Test infrastructure only."""
from __future__ import annotations

import ctypes as C

import numpy as np

from bitcaskdb_amd import _lib as L  # noqa: F401  (loads libbcw.so and with it its HIP runtime)

_hip = C.CDLL("libamdhip64.so.7")
_hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
_hip.hipFree.argtypes = [C.c_void_p]
_hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
_hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
_hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


class DevBuf:
    def __init__(self, nbytes: int, fill: int | None = 0):
        self.n = max(int(nbytes), 1)
        self.p = C.c_void_p()
        _chk(_hip.hipMalloc(C.byref(self.p), self.n), "hipMalloc")
        if fill is not None:
            _chk(_hip.hipMemset(self.p, fill, self.n), "hipMemset")

    @property
    def ptr(self) -> int:
        return int(self.p.value)

    def vp(self, off: int = 0) -> C.c_void_p:
        return C.c_void_p(self.ptr + off)

    def upload(self, data, off: int = 0):
        a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                 else data)
        _chk(_hip.hipMemcpy(self.vp(off), a.ctypes.data_as(C.c_void_p), a.nbytes, H2D), "hipMemcpy H2D")
        return self

    def download(self, nbytes: int | None = None, off: int = 0) -> np.ndarray:
        n = self.n - off if nbytes is None else int(nbytes)
        out = np.empty(max(n, 0), dtype=np.uint8)
        if n:
            _chk(_hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
            _chk(_hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), self.vp(off), n, D2H), "hipMemcpy D2H")
        return out

    def free(self):
        if self.p and self.p.value:
            _hip.hipFree(self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def sync():
    _chk(_hip.hipDeviceSynchronize(), "hipDeviceSynchronize")


def upload(data) -> DevBuf:
    a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data)
    return DevBuf(a.nbytes, fill=None).upload(a)


class DevTable:
    """a device record table (bcw_record_table) with `cap` rows"""

    def __init__(self, cap: int):
        self.cap = cap
        self.cols = {}
        ptr_t = {"u8": L.u64p, "u4": L.u32p, "u1": L.u8p}
        size = {"u8": 8, "u4": 4, "u1": 1}
        args = []
        for name, dt in L.TABLE_COLUMNS:
            b = DevBuf(max(cap, 1) * size[dt])
            self.cols[name] = (b, dt)
            args.append(C.cast(b.vp(), ptr_t[dt]))
        self.t = L.RecordTable(cap, *args)

    def column(self, name: str, n: int) -> np.ndarray:
        b, dt = self.cols[name]
        size = {"u8": 8, "u4": 4, "u1": 1}[dt]
        return b.download(n * size).view({"u8": np.uint64, "u4": np.uint32, "u1": np.uint8}[dt])
