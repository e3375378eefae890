"""Pinned host staging for the frame-ingest pipeline.

The III runner's encode is host-bound once the kernel runs near the HBM
roofline: PNG decode, TIFF deflate and -- if done naively --
pageable copies and np.stack on the submitting thread.  A StagedEncoder
keeps two batch slots, each a pinned input buffer the PNG workers decode
straight into (vcf_png_decode_rgb writes to the slot), device buffers, and a
pinned output buffer the TIFF workers read from: per batch one async H2D, one
encode launch and one async D2H on the slot's stream, while the other slot's
frames are being decoded and the previous batch's indices deflated.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import _lib
from .device import DeviceBuffer, Stream


class PinnedArray:
    """A page-locked host allocation (hipHostMalloc) viewed as a numpy array."""

    def __init__(self, shape, dtype=np.uint8):
        self.shape, self.dtype = tuple(shape), np.dtype(dtype)
        self.nbytes = int(np.prod(shape)) * self.dtype.itemsize
        p = ctypes.c_void_p()
        _lib.call("vcf_host_alloc", ctypes.byref(p), max(1, self.nbytes))
        self.ptr = p

    @property
    def array(self) -> np.ndarray:
        """The allocation as an array; every view keeps this object (and so the
        page-locked memory) alive through its ctypes base, with no reference cycle
        (device.HostBuffer.array)."""
        buf = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr.value)
        buf._owner = self
        return np.frombuffer(buf, np.uint8, count=self.nbytes).view(self.dtype).reshape(self.shape)

    def free(self):
        if self.ptr is not None and self.ptr.value:
            _lib.lib().vcf_host_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def png_probe(fn: str):
    """(H, W, natively decodable) from a PNG's signature and IHDR, or None."""
    with open(fn, "rb") as f:
        head = f.read(33)
    if len(head) < 33 or head[:8] != b"\x89PNG\r\n\x1a\n" or head[12:16] != b"IHDR":
        return None
    W, H, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", head[16:29])
    ok = interlace == 0 and ((depth == 8 and ctype in (2, 3, 6)) or (depth in (1, 2, 4) and ctype == 3))
    return H, W, ok


def decode_png_into(fn: str, out: np.ndarray) -> int:
    """Decode fn (a covered PNG) into out (H x W x 3 u8, e.g. a pinned slot); bytes read."""
    with open(fn, "rb") as f:
        data = f.read()
    _lib.call("vcf_png_decode_rgb", ctypes.c_char_p(data), len(data), out.ctypes.data_as(ctypes.c_void_p),
              out.nbytes)
    return len(data)


class StagedEncoder:
    """Two-slot pinned pipeline for encoding equal-shaped frames on one GPU."""

    def __init__(self, batch: int, H: int, W: int, out_shape, encode_launch):
        self.batch, self.H, self.W = batch, H, W
        self.out_shape = tuple(out_shape)
        self.launch = encode_launch       # (din, n, dout, stream) -> None
        fin = H * W * 3
        fout = int(np.prod(self.out_shape))
        self.slots = []
        for _ in range(2):
            self.slots.append(dict(
                hin=PinnedArray((batch, H, W, 3)), hout=PinnedArray((batch,) + self.out_shape),
                din=DeviceBuffer(batch * fin), dout=DeviceBuffer(batch * fout), stream=Stream()))

    def slot(self, b):
        return self.slots[b % 2]

    def run(self, b: int, n: int):
        """Encode the n frames of slot b%2's pinned input into its pinned output (blocking)."""
        s = self.slot(b)
        st = s["stream"]
        fin, fout = self.H * self.W * 3, int(np.prod(self.out_shape))
        _lib.call("vcf_memcpy_htod", s["din"].ptr, s["hin"].ptr, n * fin, st.handle)
        self.launch(s["din"], n, s["dout"], st)
        _lib.call("vcf_memcpy_dtoh", s["hout"].ptr, s["dout"].ptr, n * fout, st.handle)
        st.synchronize()
        return s["hout"].array[:n]

    def run_device(self, b: int, n: int):
        """Queue the encode of slot b%2's n pinned frames and leave the indices
        in HBM: -> (device output, the slot's stream); nothing is downloaded."""
        s = self.slot(b)
        st = s["stream"]
        _lib.call("vcf_memcpy_htod", s["din"].ptr, s["hin"].ptr, n * self.H * self.W * 3, st.handle)
        self.launch(s["din"], n, s["dout"], st)
        return s["dout"], st

    def close(self):
        for s in self.slots:
            for k in ("hin", "hout", "din", "dout"):
                s[k].free()
            s["stream"].close()
        self.slots = []
