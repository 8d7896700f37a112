"""Minimal device-memory helpers for GPU tests, through the HIP runtime that
libcelestia_eds.so itself links (libamdhip64.so.7). Test plumbing only: a second
runtime in the process (torch's) would not see the device once this one owns it."""
import ctypes

import numpy as np

_H2D, _D2H = 1, 2
_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        _hip.hipDeviceSynchronize.argtypes = []
        _hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        _hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        _hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        _hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p]
    return _hip


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


class DeviceBuffer:
    def __init__(self, nbytes, fill=None):
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p()
        _ck(hip().hipMalloc(ctypes.byref(self.ptr), max(self.nbytes, 1)), "hipMalloc")
        if fill is not None:
            _ck(hip().hipMemset(self.ptr, fill, self.nbytes), "hipMemset")
            # the fill runs on the null stream; the library's streams do not wait for it
            synchronize()

    def upload(self, arr):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        _ck(hip().hipMemcpy(self.ptr, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, _H2D), "H2D")

    def upload_async(self, arr, stream):
        """H2D on `stream` (ordered after the stream's earlier work); `arr` must stay alive
        until the stream is synchronized."""
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        _ck(hip().hipMemcpyAsync(self.ptr, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, _H2D, stream.ptr),
            "H2D async")
        return a

    def download(self, shape, dtype=np.uint8):
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        _ck(hip().hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), self.ptr, out.nbytes, _D2H), "D2H")
        return out

    def download_at(self, offset, shape, dtype=np.uint8):
        """D2H of shape's bytes starting `offset` bytes into the buffer."""
        out = np.empty(shape, dtype)
        assert offset + out.nbytes <= self.nbytes
        src = ctypes.c_void_p(self.ptr.value + offset)
        _ck(hip().hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), src, out.nbytes, _D2H), "D2H")
        return out

    def free(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        self.ptr = ctypes.c_void_p()
        _ck(hip().hipStreamCreate(ctypes.byref(self.ptr)), "hipStreamCreate")

    def synchronize(self):
        _ck(hip().hipStreamSynchronize(self.ptr), "hipStreamSynchronize")

    def __del__(self):
        try:
            if self.ptr:
                hip().hipStreamDestroy(self.ptr)
        except Exception:
            pass


def synchronize():
    _ck(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
