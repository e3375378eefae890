"""CBAAC entropy coding (src/CBAAC.py) through libvcf_amd.so's native coder.

compress(ndarray) -> BytesIO and decompress(bytes) -> uint8 ndarray with the
reference's container: uint32 ndims, uint32 shape[ndims] (native little
endian), then the arithmetic-coded bit stream (CBAAC.py:81-112)."""
from __future__ import annotations

import ctypes
import io

import numpy as np

from . import _lib as L

FILE_EXTENSION = ".adpt_arith"   # CBAAC.py:75


def encode_symbols(sym: np.ndarray, order: int = 0) -> bytes:
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    cap = int(L.lib().vcf_cbaac_bound(sym.size))
    out = np.empty(cap, np.uint8)
    nb, nbits = ctypes.c_int64(), ctypes.c_int64()
    L.call("vcf_cbaac_encode", sym.ctypes.data, sym.size, int(order), out.ctypes.data, cap,
           ctypes.byref(nb), ctypes.byref(nbits))
    return out[:nb.value].tobytes()


def decode_symbols(data: bytes, n: int, order: int = 0) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8)
    out = np.empty(n, np.uint8)
    L.call("vcf_cbaac_decode", buf.ctypes.data if buf.size else None, buf.size, int(n), int(order),
           out.ctypes.data)
    return out


def model_trace(sym: np.ndarray, order: int = 0) -> np.ndarray:
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    t = np.empty((sym.size, 3), np.int32)
    L.call("vcf_cbaac_model_trace", sym.ctypes.data, sym.size, int(order), t.ctypes.data)
    return t


class CBAACCodec:
    """The entropy stage of CBAAC.CoDec (CBAAC.py:72-156)."""

    file_extension = FILE_EXTENSION

    def __init__(self, order: int = 0):
        self.ORDER = int(order)

    def compress(self, img: np.ndarray, fn=None) -> io.BytesIO:
        img = np.asarray(img)
        b = io.BytesIO()
        b.write(np.array([img.ndim], np.uint32).tobytes())
        b.write(np.array(img.shape, np.uint32).tobytes())
        # flatten().astype(int32) -> symbols; the model has 256 symbols, so
        # the values must be bytes (the reference's callers pass uint8)
        flat = img.ravel()
        if flat.dtype != np.uint8:   # (uint8 input, the callers' case, needs no check or copy)
            if flat.size and (flat.min() < 0 or flat.max() > 255):
                raise ValueError("CBAAC codes byte symbols (0..255)")
            flat = flat.astype(np.uint8)
        b.write(encode_symbols(flat, self.ORDER))
        b.seek(0)
        return b

    def decompress(self, data, fn=None) -> np.ndarray:
        if isinstance(data, io.BytesIO):
            data = data.getvalue()
        data = bytes(data)
        try:
            nd = int(np.frombuffer(data[:4], np.uint32)[0])
            shape = tuple(int(v) for v in np.frombuffer(data[4:4 + 4 * nd], np.uint32))
        except Exception:
            return np.zeros((10, 10), np.uint8)    # CBAAC.py:101-102
        n = int(np.prod(shape))
        return decode_symbols(data[4 + 4 * nd:], n, self.ORDER).reshape(shape)

    # the reference's public names (CBAAC.py:81, :97; compress/decompress wrap them, :152-156)
    def compress_fn(self, img, fn):
        return self.compress(img, fn)

    def decompress_fn(self, compressed_bytes, fn):
        return self.decompress(compressed_bytes, fn)
