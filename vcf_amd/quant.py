"""Deadzone quantizer plug-in on the GPU (deadzone.py:95-117, assumption A5).

deadzone_quantize(x, Q)   -> int32 indices, (x / Q) truncated toward zero;
deadzone_dequantize(k, Q) -> Q * k in k's dtype (int16 or int32, wrapping).
Host arrays in, host arrays out; the arithmetic runs in libvcf_amd.so
(vcf_deadzone_quantize / vcf_deadzone_dequantize).  There is no CPU path.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .device import DeviceBuffer

_DTYPES = {np.dtype(np.float32): L.VCF_DTYPE_F32, np.dtype(np.float64): L.VCF_DTYPE_F64,
           np.dtype(np.int16): L.VCF_DTYPE_I16, np.dtype(np.int32): L.VCF_DTYPE_I32,
           np.dtype(np.uint8): L.VCF_DTYPE_U8}


def deadzone_quantize(x: np.ndarray, Q: int) -> np.ndarray:
    x = np.ascontiguousarray(x)
    if x.dtype not in _DTYPES:
        raise TypeError(f"unsupported dtype {x.dtype}")
    out = np.empty(x.shape, np.int32)
    if x.size == 0:
        return out
    dx, dk = DeviceBuffer.from_array(x), DeviceBuffer(out.nbytes)
    try:
        L.call("vcf_deadzone_quantize", dx.ptr, _DTYPES[x.dtype], x.size, int(Q), dk.ptr, None)
        return dk.download(out)
    finally:
        dx.free()
        dk.free()


def deadzone_dequantize(k: np.ndarray, Q: int) -> np.ndarray:
    k = np.ascontiguousarray(k)
    if k.dtype not in (np.int16, np.int32):
        raise TypeError(f"unsupported index dtype {k.dtype}")
    out = np.empty_like(k)
    if k.size == 0:
        return out
    dk, dy = DeviceBuffer.from_array(k), DeviceBuffer(out.nbytes)
    try:
        L.call("vcf_deadzone_dequantize", dk.ptr, _DTYPES[k.dtype], k.size, int(Q), dy.ptr, None)
        return dy.download(out)
    finally:
        dk.free()
        dy.free()
