"""CBAHC entropy coding (src/CBAHC.py) through libvcf_amd.so's native coder.

compress(ndarray, fn) -> BytesIO holding the bit stream, plus the side file
{fn}_adaptive_huffman_tree.pkl.gz = gzip(np.save(shape) + pickle({"order",
"nbits"})) as the reference writes it (CBAHC.py:169-221); decompress(bytes,
fn) reads both back (:226-276).  The side file is read with np.load
(allow_pickle=False) and an unpickler that refuses every global."""
from __future__ import annotations

import ctypes
import gzip
import io
import pickle

import numpy as np

from . import _lib as L

FILE_EXTENSION = ".huf"   # CBAHC.py:163


def encode_symbols(sym: np.ndarray, order: int = 0):
    """-> (bytes, nbits)."""
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    cap = int(L.lib().vcf_cbahc_bound(sym.size))
    out = np.empty(cap, np.uint8)
    nb, nbits = ctypes.c_int64(), ctypes.c_int64()
    L.call("vcf_cbahc_encode", sym.ctypes.data, sym.size, int(order), out.ctypes.data, cap,
           ctypes.byref(nb), ctypes.byref(nbits))
    return out[:nb.value].tobytes(), nbits.value


def decode_symbols(data: bytes, nbits: int, n: int, order: int = 0) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8)
    out = np.empty(n, np.uint8)
    L.call("vcf_cbahc_decode", buf.ctypes.data if buf.size else None, int(nbits), int(n), int(order),
           out.ctypes.data)
    return out


class _NoGlobals(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"refusing global {module}.{name}")


def _side_file(fn):
    return f"{fn}_adaptive_huffman_tree.pkl.gz"


class CBAHCCodec:
    """The entropy stage of CBAHC.CoDec (CBAHC.py:158-283)."""

    file_extension = FILE_EXTENSION

    def __init__(self, order: int = 0):
        if int(order) < 0:
            raise ValueError("order must be >= 0")
        self.order = int(order)

    def compress(self, img, fn="/tmp/encoded") -> io.BytesIO:
        img = np.asarray(img)
        data, nbits = encode_symbols(img.astype(np.uint8), self.order)
        with gzip.open(_side_file(fn), "wb") as f:
            np.save(f, img.shape)
            pickle.dump({"order": self.order, "nbits": nbits}, f)
        return io.BytesIO(data)

    def decompress(self, data, fn="/tmp/encoded") -> np.ndarray:
        if isinstance(data, io.BytesIO):
            data = data.getvalue()
        with gzip.open(_side_file(fn), "rb") as f:
            shape = tuple(int(v) for v in np.load(f, allow_pickle=False))
            meta = _NoGlobals(f).load()
        n = int(np.prod(shape))
        return decode_symbols(bytes(data), int(meta["nbits"]), n, int(meta["order"])).reshape(shape)

    # the reference's public names (CBAHC.py:169, :226; compress/decompress wrap them, :223, :278)
    def compress_fn(self, img, fn):
        return self.compress(img, fn)

    def decompress_fn(self, compressed_img, fn):
        return self.decompress(compressed_img, fn)
