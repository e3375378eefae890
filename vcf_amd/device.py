"""Device memory, streams and events over the C ABI (no PyTorch)."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call, lib


def device_count() -> int:
    n = ctypes.c_int(0)
    call("vcf_device_count", ctypes.byref(n))
    return n.value


def set_device(dev: int) -> None:
    call("vcf_set_device", dev)


def synchronize() -> None:
    call("vcf_device_sync")


class Stream:
    def __init__(self):
        p = ctypes.c_void_p()
        call("vcf_stream_create", ctypes.byref(p))
        self.handle = p

    def synchronize(self) -> None:
        call("vcf_stream_sync", self.handle)

    def wait_event(self, event: "Event") -> None:
        """Later work on this stream waits for `event`."""
        call("vcf_stream_wait_event", self.handle, event.handle)

    def close(self) -> None:
        if self.handle is not None and self.handle.value:
            lib().vcf_stream_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _h(stream) -> ctypes.c_void_p:
    return stream.handle if isinstance(stream, Stream) else ctypes.c_void_p(stream or 0)


class Event:
    def __init__(self):
        p = ctypes.c_void_p()
        call("vcf_event_create", ctypes.byref(p))
        self.handle = p

    def record(self, stream=None) -> None:
        call("vcf_event_record", self.handle, _h(stream))

    def synchronize(self) -> None:
        call("vcf_event_sync", self.handle)

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        call("vcf_event_elapsed_ms", self.handle, end.handle, ctypes.byref(ms))
        return ms.value

    def __del__(self):
        try:
            if self.handle is not None and self.handle.value:
                lib().vcf_event_destroy(self.handle)
        except Exception:
            pass


class DeviceBuffer:
    """A caller-owned HBM allocation (hipMalloc)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        call("vcf_malloc", ctypes.byref(p), max(1, self.nbytes))
        self.ptr = p

    @classmethod
    def from_array(cls, arr: np.ndarray, stream=None) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        b.upload(arr, stream)
        return b

    def address(self, offset: int = 0) -> ctypes.c_void_p:
        return ctypes.c_void_p(self.ptr.value + offset)

    def upload(self, arr: np.ndarray, stream=None, offset: int = 0) -> None:
        arr = np.ascontiguousarray(arr)
        if arr.nbytes + offset > self.nbytes:
            raise ValueError("upload larger than the buffer")
        call("vcf_memcpy_htod", self.address(offset), arr.ctypes.data_as(ctypes.c_void_p),
             arr.nbytes, _h(stream))
        if stream is None:
            call("vcf_stream_sync", ctypes.c_void_p(0))

    def download(self, out: np.ndarray, stream=None, offset: int = 0) -> np.ndarray:
        if not out.flags.c_contiguous:
            raise ValueError("download target must be C-contiguous")
        if out.nbytes + offset > self.nbytes:
            raise ValueError("download larger than the buffer")
        call("vcf_memcpy_dtoh", out.ctypes.data_as(ctypes.c_void_p), self.address(offset),
             out.nbytes, _h(stream))
        if stream is None:
            call("vcf_stream_sync", ctypes.c_void_p(0))
        return out

    def fill(self, value: int, stream=None) -> None:
        call("vcf_memset", self.ptr, value, self.nbytes, _h(stream))

    def free(self) -> None:
        if self.ptr is not None and self.ptr.value:
            lib().vcf_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_dtod(dst: DeviceBuffer, dst_off: int, src: DeviceBuffer, src_off: int, nbytes: int, stream=None) -> None:
    """nbytes from src[src_off:] to dst[dst_off:], enqueued on `stream`."""
    if nbytes <= 0:
        return
    if dst_off + nbytes > dst.nbytes or src_off + nbytes > src.nbytes:
        raise ValueError("device copy out of bounds")
    call("vcf_memcpy_dtod", dst.address(dst_off), src.address(src_off), int(nbytes), _h(stream))


class HostBuffer:
    """Page-locked host memory (hipHostMalloc): full-speed copies to and from
    the device; `array` is a uint8 view."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        call("vcf_host_alloc", ctypes.byref(p), max(1, self.nbytes))
        self.ptr = p

    @property
    def array(self) -> np.ndarray:
        """A uint8 view of the buffer.  Every view (and its slices and memoryviews)
        keeps this HostBuffer alive through its ctypes base, so the page-locked memory
        is freed only after the last view is gone -- a view that outlived its buffer
        read freed memory (bench.py's C5 check after the block had returned).  The
        buffer holds no view itself, so there is no reference cycle."""
        cbuf = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr.value)
        cbuf._owner = self
        return np.ctypeslib.as_array(cbuf)[:self.nbytes]

    def free(self) -> None:
        if self.ptr is not None and self.ptr.value:
            lib().vcf_host_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_pieces(src: DeviceBuffer, table: DeviceBuffer, n_pieces: int, dst: DeviceBuffer, stream=None) -> None:
    """n_pieces device copies in one launch (vcf_copy_pieces): table = int64
    (src offset, dst offset, bytes) triples in device memory."""
    call("vcf_copy_pieces", src.ptr, table.ptr, int(n_pieces), dst.ptr, _h(stream))
