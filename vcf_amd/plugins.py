"""The YCrCb and LloydMax plug-ins on the GPU.

YCrCb (src/YCrCb.py:25-72): ycrcb_dz_encode / ycrcb_dz_decode run the
stand-alone pixel codec's span between reading the image and the entropy
codec in one kernel each (vcf_ycrcb_dz_*); ycrcb_from_rgb / ycrcb_to_rgb
are the colour transform alone (for the LloydMax quantizer).  The
transform is OpenCV's integer RGB<->YCrCb (assumption A12, unpinned).

LloydMax (src/LloydMax.py:75-143): lm_quantize_device runs, per channel,
numpy.histogram (vcf_lm_histogram), the glue's +1, the Lloyd-Max design
(vcf_lm_design, host, A13 unpinned) and the encoder (vcf_lm_encode);
lm_dequantize_device the centroid lookup (vcf_lm_decode).  There is no CPU
path: the arithmetic runs in libvcf_amd.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from ._lib import call
from .device import DeviceBuffer, _h

DTYPES = {np.dtype(np.uint8): L.VCF_DTYPE_U8, np.dtype(np.int16): L.VCF_DTYPE_I16,
          np.dtype(np.uint16): L.VCF_DTYPE_U16, np.dtype(np.float32): L.VCF_DTYPE_F32}


def _code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt not in DTYPES:
        raise TypeError(f"unsupported dtype {dt}")
    return DTYPES[dt]


def _rgb(a: np.ndarray, what: str) -> np.ndarray:
    a = np.ascontiguousarray(a)
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"{what} must be H x W x 3")
    return a


# ---- YCrCb -------------------------------------------------------------------
def _px_map(fn: str, a: np.ndarray, out_dtype) -> np.ndarray:
    out = np.empty(a.shape, out_dtype)
    n_px = a.shape[0] * a.shape[1]
    if n_px == 0:
        return out
    din, dout = DeviceBuffer.from_array(a), DeviceBuffer(out.nbytes)
    try:
        call(fn, din.ptr, n_px, dout.ptr, None)
        return dout.download(out)
    finally:
        din.free()
        dout.free()


def ycrcb_from_rgb(rgb: np.ndarray) -> np.ndarray:
    """color_transforms.YCrCb.from_RGB (A12) on a u8 H x W x 3 frame."""
    rgb = _rgb(rgb, "rgb")
    if rgb.dtype != np.uint8:
        raise TypeError("from_RGB takes uint8 frames")
    return _px_map("vcf_ycrcb_from_rgb", rgb, np.uint8)


def ycrcb_to_rgb(ycc: np.ndarray) -> np.ndarray:
    """color_transforms.YCrCb.to_RGB (A12) on a u8 H x W x 3 frame."""
    ycc = _rgb(ycc, "ycrcb")
    if ycc.dtype != np.uint8:
        raise TypeError("to_RGB takes uint8 frames")
    return _px_map("vcf_ycrcb_to_rgb", ycc, np.uint8)


def ycrcb_dz_encode(rgb: np.ndarray, Q: int) -> np.ndarray:
    """YCrCb.encode (:33-51) with -a deadzone: u8 RGB -> uint16 indices."""
    rgb = _rgb(rgb, "rgb")
    if rgb.dtype != np.uint8:
        raise TypeError("rgb must be uint8")
    out = np.empty(rgb.shape, np.uint16)
    n_px = rgb.shape[0] * rgb.shape[1]
    if n_px == 0:
        call("vcf_ycrcb_dz_encode", None, 0, int(Q), None, None)
        return out
    din, dout = DeviceBuffer.from_array(rgb), DeviceBuffer(out.nbytes)
    try:
        call("vcf_ycrcb_dz_encode", din.ptr, n_px, int(Q), dout.ptr, None)
        return dout.download(out)
    finally:
        din.free()
        dout.free()


def ycrcb_dz_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """YCrCb.decode (:53-72) with -a deadzone: uint16 indices -> u8 RGB."""
    k = _rgb(k, "k")
    if k.dtype != np.uint16:
        raise TypeError("k must be uint16 (YCrCb.py:46)")
    out = np.empty(k.shape, np.uint8)
    n_px = k.shape[0] * k.shape[1]
    if n_px == 0:
        call("vcf_ycrcb_dz_decode", None, 0, int(Q), None, None)
        return out
    din, dout = DeviceBuffer.from_array(k), DeviceBuffer(out.nbytes)
    try:
        call("vcf_ycrcb_dz_decode", din.ptr, n_px, int(Q), dout.ptr, None)
        return dout.download(out)
    finally:
        din.free()
        dout.free()


# ---- YCoCg.py and deadzone.py, the stand-alone pixel codecs --------------------
def _map(fn: str, a: np.ndarray, out_dtype, n: int, Q: int) -> np.ndarray:
    out = np.empty(a.shape, out_dtype)
    if n == 0:
        call(fn, None, 0, int(Q), None, None)   # argument checks only
        return out
    din, dout = DeviceBuffer.from_array(a), DeviceBuffer(out.nbytes)
    try:
        call(fn, din.ptr, n, int(Q), dout.ptr, None)
        return dout.download(out)
    finally:
        din.free()
        dout.free()


def ycocg_dz_encode(rgb: np.ndarray, Q: int) -> np.ndarray:
    """YCoCg.encode (src/YCoCg.py:33-56) with -a deadzone: u8 RGB -> uint16 indices."""
    rgb = _rgb(rgb, "rgb")
    if rgb.dtype != np.uint8:
        raise TypeError("rgb must be uint8")
    return _map("vcf_ycocg_dz_encode", rgb, np.uint16, rgb.shape[0] * rgb.shape[1], Q)


def ycocg_dz_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """YCoCg.decode (:58-85) with -a deadzone: uint16 indices -> u8 RGB."""
    k = _rgb(k, "k")
    if k.dtype != np.uint16:
        raise TypeError("k must be uint16 (YCoCg.py:50)")
    return _map("vcf_ycocg_dz_decode", k, np.uint8, k.shape[0] * k.shape[1], Q)


def dz_u8_encode(img: np.ndarray, Q: int) -> np.ndarray:
    """deadzone.encode (src/deadzone.py:67-79): u8 image -> u8 indices (any shape)."""
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8:
        raise TypeError("img must be uint8")
    return _map("vcf_dz_u8_encode", img, np.uint8, img.size, Q)


def dz_u8_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """deadzone.decode (:81-93): u8 indices -> Q * k in uint8."""
    k = np.ascontiguousarray(k)
    if k.dtype != np.uint8:
        raise TypeError("k must be uint8 (deadzone.py:76)")
    return _map("vcf_dz_u8_decode", k, np.uint8, k.size, Q)


# ---- LloydMax ----------------------------------------------------------------
def lm_levels(Q: int, min_val: int, max_val: int) -> int:
    return call("vcf_lm_levels", int(Q), int(min_val), int(max_val))


def lm_histogram_device(x: DeviceBuffer, dtype, n_px: int, channels: int, min_val: int, max_val: int,
                        stream=None) -> np.ndarray:
    """numpy.histogram(x[..., c], bins=max-min+1, range=(min, max))[0] per channel -> (C, L) int64."""
    nb = int(max_val) - int(min_val) + 1
    if nb < 1:
        raise ValueError("max must be larger than min in range parameter.")
    counts = DeviceBuffer(channels * nb * 8)
    try:
        call("vcf_lm_histogram", x.ptr if n_px else None, _code(dtype), int(n_px), int(channels), int(min_val),
             int(max_val), counts.ptr, _h(stream))
        out = np.empty((channels, nb), np.int64)
        counts.download(out, stream)
        if stream is not None:
            stream.synchronize()
        return out
    finally:
        counts.free()


def lm_design(counts: np.ndarray, Q: int, min_val: int) -> np.ndarray:
    """LloydMax_Quantizer(Q_step=Q, counts, min_val, ...).get_representation_levels() (A13)."""
    c = np.ascontiguousarray(counts, dtype=np.int64)
    n_bins = c.shape[0]
    cent = np.empty(-(-n_bins // int(Q)) if Q >= 1 else 1, np.float64)
    n = call("vcf_lm_design", c.ctypes.data_as(ctypes.c_void_p), n_bins, int(Q), int(min_val),
             cent.ctypes.data_as(ctypes.c_void_p))
    return cent[:n]


def lm_quantize_device(x: DeviceBuffer, dtype, n_px: int, channels: int, Q: int, min_val: int, max_val: int,
                       k_dtype, out: DeviceBuffer | None = None, stream=None):
    """LloydMax.quantize_fn (:75-114) on device data: (k DeviceBuffer in k_dtype, [centroids per channel])."""
    N = lm_levels(Q, min_val, max_val)
    hist = lm_histogram_device(x, dtype, n_px, channels, min_val, max_val, stream)
    cents = [lm_design(hist[c] + 1, Q, min_val) for c in range(channels)]   # :101 histogram_img += 1
    ksz = np.dtype(k_dtype).itemsize
    if out is None:
        out = DeviceBuffer(n_px * channels * ksz)
    elif out.nbytes < n_px * channels * ksz:
        raise ValueError("output buffer too small")
    if n_px:
        dc = DeviceBuffer.from_array(np.stack(cents), stream)
        try:
            call("vcf_lm_encode", x.ptr, _code(dtype), int(n_px), int(channels), dc.ptr, N, out.ptr,
                 _code(k_dtype), _h(stream))
            if stream is not None:
                stream.synchronize()
        finally:
            dc.free()
    return out, cents


def lm_dequantize_device(k: DeviceBuffer, k_dtype, n_px: int, channels: int, cents, y_dtype,
                         out: DeviceBuffer | None = None, stream=None) -> DeviceBuffer:
    """LloydMax.dequantize_fn (:116-143): y = empty_like(k); y[..., c] = centroids_c[k[..., c]]."""
    cents = [np.asarray(c, np.float64) for c in cents]
    N = len(cents[0])
    if any(len(c) != N for c in cents) or len(cents) != channels:
        raise ValueError("one centroid table of the same length per channel")
    ysz = np.dtype(y_dtype).itemsize
    if out is None:
        out = DeviceBuffer(n_px * channels * ysz)
    if not n_px:
        return out
    dc = DeviceBuffer.from_array(np.stack(cents), stream)
    bad = DeviceBuffer(4)
    try:
        bad.fill(0, stream)
        call("vcf_lm_decode", k.ptr, _code(k_dtype), int(n_px), int(channels), dc.ptr, N, out.ptr,
             _code(y_dtype), bad.ptr, _h(stream))
        flag = bad.download(np.zeros(1, np.int32), stream)
        if stream is not None:
            stream.synchronize()
        if flag[0]:
            raise IndexError(f"index out of bounds for the {N} representation levels")
        return out
    finally:
        dc.free()
        bad.free()


def lm_quantize(img: np.ndarray, Q: int, min_val: int = 0, max_val: int = 255):
    """Host convenience: H x W x C array -> (k in img's dtype, [centroids])  (k = empty_like(img), :96)."""
    a = np.ascontiguousarray(img)
    if a.ndim == 2:
        a = a[:, :, None]
    n_px, C = a.shape[0] * a.shape[1], a.shape[2]
    dx = DeviceBuffer.from_array(a)
    try:
        dk, cents = lm_quantize_device(dx, a.dtype, n_px, C, Q, min_val, max_val, a.dtype)
        k = dk.download(np.empty(a.shape, a.dtype))
        dk.free()
    finally:
        dx.free()
    return (k if np.asarray(img).ndim == 3 else k[:, :, 0]), cents


def lm_dequantize(k: np.ndarray, cents) -> np.ndarray:
    """Host convenience: y = empty_like(k); y[..., c] = centroids_c[k[..., c]] (truncated)."""
    a = np.ascontiguousarray(k)
    if a.ndim == 2:
        a = a[:, :, None]
    n_px, C = a.shape[0] * a.shape[1], a.shape[2]
    dk = DeviceBuffer.from_array(a)
    try:
        dy = lm_dequantize_device(dk, a.dtype, n_px, C, cents, a.dtype)
        y = dy.download(np.empty(a.shape, a.dtype))
        dy.free()
    finally:
        dk.free()
    return y if np.asarray(k).ndim == 3 else y[:, :, 0]
