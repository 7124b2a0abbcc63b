"""Device buffers for kp_score_dev callers (tests, bench), allocated through the
SAME HIP runtime libkplace is bound to. libkplace needs `libamdhip64.so.7`: in a
process that imported torch first that soname is torch's bundled runtime, else
/opt/rocm's (two HIP runtimes in one process do not share a device). Loading
libkplace first and then asking the loader for the soname returns whichever one
it got."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_hip = None


def hip() -> C.CDLL:
    global _hip
    if _hip is None:
        from . import _abi
        _abi.load_library(os.environ.get("KPLACE_LIB") or None)  # binds libamdhip64.so.7
        try:
            _hip = C.CDLL("libamdhip64.so.7")  # the loaded one (soname match)
        except OSError:
            rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
            _hip = C.CDLL(os.path.join(rocm, "lib", "libamdhip64.so.7"))
        _hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        _hip.hipFree.argtypes = [C.c_void_p]
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        _hip.hipSetDevice.argtypes = [C.c_int]
    return _hip


class DeviceBuffer:
    """hipMalloc'd bytes on `device`; .ptr is the device address."""

    def __init__(self, nbytes: int, device: int = 0, fill: int | None = None):
        h = hip()
        if h.hipSetDevice(device) != 0:
            raise RuntimeError("hipSetDevice failed")
        p = C.c_void_p()
        if h.hipMalloc(C.byref(p), max(int(nbytes), 1)) != 0:
            raise MemoryError(f"hipMalloc of {nbytes} bytes failed")
        self.ptr, self.nbytes = p.value, int(nbytes)
        if fill is not None and h.hipMemset(self.ptr, fill, self.nbytes) != 0:
            raise RuntimeError("hipMemset failed")

    def to_numpy(self, dtype, shape, offset: int = 0) -> np.ndarray:
        """Bytes [offset, offset + size) of the buffer as an array."""
        out = np.empty(shape, dtype)
        if offset < 0 or offset + out.nbytes > self.nbytes:
            raise ValueError("buffer smaller than the requested array")
        if hip().hipMemcpy(out.ctypes.data, self.ptr + offset, out.nbytes, 2) != 0:  # DeviceToHost
            raise RuntimeError("hipMemcpy failed")
        return out

    def close(self) -> None:
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
