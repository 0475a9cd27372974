"""ctypes binding of the C-ABI in include/nimble_amd.h (libnimble_amd.so).

The product path has no CPU fallback: if the HIP library is missing or no
ROCm device is present, calls raise instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnimble_amd.so")

_lib = None


class NativeLibraryMissing(ImportError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        L.nimble_world_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.nimble_world_create.restype = C.c_int
        L.nimble_world_destroy.argtypes = [C.c_void_p]
        L.nimble_world_destroy.restype = C.c_int
        L.nimble_snapshot_doubles.argtypes = [C.c_void_p]
        L.nimble_snapshot_doubles.restype = C.c_int64
        L.nimble_lcp_cache_doubles.argtypes = [C.c_void_p]
        L.nimble_lcp_cache_doubles.restype = C.c_int64
        L.nimble_forward.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 5 + [C.c_void_p]
        L.nimble_forward.restype = C.c_int
        L.nimble_backward.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6 + [C.c_void_p]
        L.nimble_backward.restype = C.c_int
        L.nimble_last_error.argtypes = []
        L.nimble_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"nimble_amd error {rc}: {lib().nimble_last_error().decode()}")


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("nimblephysics_amd runs on the ROCm device only; got a CPU tensor")
        if t is not None and t.dtype.is_floating_point and str(t.dtype) != "torch.float64":
            raise TypeError("nimblephysics_amd computes in float64 (the reference's s_t); got " + str(t.dtype))


class DeviceWorld:
    """A world model uploaded to the device (nimble_world_create)."""

    def __init__(self, world):
        L = lib()
        desc, keep = world.desc()
        self._keep = keep
        h = C.c_void_p()
        _check(L.nimble_world_create(C.byref(desc), C.byref(h)))
        self.h = h
        self.n = world.getNumDofs()
        self.snapshot_doubles = int(L.nimble_snapshot_doubles(h))
        self.cache_doubles = int(L.nimble_lcp_cache_doubles(h))

    def close(self):
        if self.h:
            lib().nimble_world_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, state, forces, lcp_cache, next_state, snapshot, stream_ptr: int):
        _require_device(state, forces, lcp_cache, next_state, snapshot)
        B = state.shape[0]
        _check(lib().nimble_forward(self.h, B, _ptr(state), _ptr(forces), _ptr(lcp_cache), _ptr(next_state),
                                    _ptr(snapshot), C.c_void_p(stream_ptr)))

    def backward(self, state, forces, snapshot, grad_next, grad_state, grad_forces, stream_ptr: int):
        _require_device(state, forces, snapshot, grad_next, grad_state, grad_forces)
        B = state.shape[0]
        _check(lib().nimble_backward(self.h, B, _ptr(state), _ptr(forces), _ptr(snapshot), _ptr(grad_next),
                                     _ptr(grad_state), _ptr(grad_forces), C.c_void_p(stream_ptr)))
