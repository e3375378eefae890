"""CPU restatement of the §8(f) row-4 plug-ins -- TEST INFRASTRUCTURE ONLY
(tests/, __graft_entry__.smoke(), bench.py's cpu_baseline); the product never
imports it.

* YCrCb.py (src/YCrCb.py:25-72): the stand-alone pixel codec.  Its colour
  transform is color_transforms.YCrCb (un-vendored), assumed to be OpenCV's
  integer RGB<->YCrCb (A12, tests/golden/shims/color_transforms/YCrCb.py).
* LloydMax.py (src/LloydMax.py:75-143): numpy.histogram of each channel with
  bins = max_val - min_val + 1 over range=(min_val, max_val) (restated from
  numpy 1.26, the reference's numpy: lib/histograms.py's uniform-bin path),
  +1, and scalar_quantization's LloydMax_Quantizer (un-vendored), assumed to
  be the textbook Lloyd-Max design of tests/golden/shims/scalar_quantization/
  LloydMax_quantization.py (A13).

Parity: the glue is pinned by tests/golden/plug_*.npz (the reference's own
modules run under python3.9 with those shims, make_golden_plugins.py); the
A12/A13 arithmetic is unpinned (neither package nor OpenCV is available).
"""
from __future__ import annotations

import math

import numpy as np

MAX_ITERS = 100


# ---- A12: OpenCV RGB<->YCrCb on uint8 (yuv_shift 14, CV_DESCALE, saturate) ----
def ycrcb_from_rgb(rgb: np.ndarray) -> np.ndarray:
    a = np.asarray(rgb).astype(np.int64)
    r, g, b = a[..., 0], a[..., 1], a[..., 2]
    y = (r * 4899 + g * 9617 + b * 1868 + 8192) >> 14
    cr = ((r - y) * 11682 + (128 << 14) + 8192) >> 14
    cb = ((b - y) * 9241 + (128 << 14) + 8192) >> 14
    return np.clip(np.stack([y, cr, cb], -1), 0, 255).astype(np.uint8)


def ycrcb_to_rgb(ycrcb: np.ndarray) -> np.ndarray:
    a = np.asarray(ycrcb).astype(np.int64)
    y, cr, cb = a[..., 0], a[..., 1] - 128, a[..., 2] - 128
    r = y + ((cr * 22987 + 8192) >> 14)
    g = y + ((cb * -5636 + cr * -11698 + 8192) >> 14)
    b = y + ((cb * 29049 + 8192) >> 14)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


# ---- numpy 1.26 histogram(x, bins=n, range=(lo, hi)), uniform-bin path ----
def histogram(x: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Counts (int64) of numpy.histogram(x, bins=hi-lo+1, range=(lo, hi)) as numpy 1.26
    computes them: bin_type = result_type(lo, hi, x) under value-based casting (float32
    for float32 data, float64 for integer data), edges = linspace(lo, hi, n+1) in that
    type, index estimate ((x - lo) / (hi - lo)) * n truncated, then corrected once
    against the edges (the last bin includes hi)."""
    x = np.asarray(x).ravel()
    n = hi - lo + 1
    T = np.float32 if x.dtype == np.float32 else np.float64
    keep = (x >= lo) & (x <= hi)
    a = x[keep].astype(T)
    step = (hi - lo) / (n)                      # linspace: delta / div in float64
    edges = (np.arange(n + 1, dtype=np.float64) * step + lo)
    edges[-1] = hi
    edges = edges.astype(T)
    f = ((a - T(lo)) / T(hi - lo)) * T(n)
    idx = f.astype(np.int64)
    idx[idx == n] -= 1
    dec = a < edges[idx]
    idx[dec] -= 1
    inc = (a >= edges[idx + 1]) & (idx != n - 1)
    idx[inc] += 1
    return np.bincount(idx, minlength=n).astype(np.int64)


# ---- A13: Lloyd-Max design over an integer histogram ----
def levels(Q: int, lo: int, hi: int) -> int:
    L = hi - lo + 1
    return -(-L // Q)


def lloydmax_design(counts: np.ndarray, Q: int, lo: int) -> np.ndarray:
    counts = np.asarray(counts).astype(np.int64)
    L = counts.shape[0]
    N = -(-L // Q)
    v = np.arange(lo, lo + L, dtype=np.int64)
    S0 = np.concatenate([[0], np.cumsum(counts)])
    S1 = np.concatenate([[0], np.cumsum(counts * v)])

    def cent(b):
        return np.array([float(S1[b[j + 1]] - S1[b[j]]) / float(S0[b[j + 1]] - S0[b[j]]) for j in range(N)])

    b = [j * Q for j in range(N)] + [L]
    for _ in range(MAX_ITERS):
        c = cent(b)
        nb = [0] + [math.ceil((c[j - 1] + c[j]) / 2) - lo for j in range(1, N)] + [L]
        if nb == b:
            break
        b = nb
    return cent(b)


def lm_encode(x: np.ndarray, centroids: np.ndarray) -> np.ndarray:
    c = np.asarray(centroids, np.float64)
    return np.searchsorted((c[:-1] + c[1:]) / 2, np.asarray(x).astype(np.float64), side="right")


def lm_quantize(img: np.ndarray, Q: int, lo: int, hi: int):
    """LloydMax.quantize_fn (:75-114): per channel -> (k in img's dtype, [centroids])."""
    k = np.empty_like(img)
    cents = []
    for c in range(img.shape[2]):
        counts = histogram(img[..., c], lo, hi) + 1
        cent = lloydmax_design(counts, Q, lo)
        cents.append(cent)
        k[..., c] = lm_encode(img[..., c], cent)
    return k, cents


def lm_dequantize(k: np.ndarray, cents) -> np.ndarray:
    """LloydMax.dequantize_fn (:120-143): y = empty_like(k); y[..., c] = centroids[k]."""
    y = np.empty_like(k)
    for c in range(k.shape[2]):
        y[..., c] = np.asarray(cents[c])[k[..., c].astype(np.int64)]
    return y


# ---- the stand-alone codecs' index arrays (before the entropy codec) ----
def ycrcb_dz_encode(rgb: np.ndarray, Q: int) -> np.ndarray:
    """YCrCb.encode (:33-51) with -a deadzone: from_RGB, int16, + [0,0,0], (x/Q).astype(int32), uint16."""
    x = ycrcb_from_rgb(rgb).astype(np.int16)
    return (x / Q).astype(np.int32).astype(np.uint16)


def ycrcb_dz_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """YCrCb.decode (:53-72): Q*k in uint16, int16, uint8, to_RGB, clip."""
    # numpy 1.26: uint16 array * int -> uint16 (wrapping) for Q < 2**16, a wider type otherwise;
    # either way the uint8 cast keeps the low byte of Q * k
    y = ((np.asarray(k, np.uint16).astype(np.int64) * int(Q)) & 0xFFFF).astype(np.uint16)
    y = y.astype(np.int16).astype(np.uint8)
    return ycrcb_to_rgb(y)


# ---- YCoCg.py / deadzone.py as stand-alone codecs (A4, A5) ----
def ycocg_i16(rgb: np.ndarray) -> np.ndarray:
    """YCoCg.encode (src/YCoCg.py:36-38): img.astype(int16), then color_transforms.YCoCg.from_RGB
    (A4: the float64 matrix products stored into empty_like(int16), i.e. truncated toward zero)."""
    a = np.asarray(rgb).astype(np.int16)
    R, G, B = a[..., 0], a[..., 1], a[..., 2]
    o = np.empty_like(a)
    o[..., 0] = R / 4 + G / 2 + B / 4
    o[..., 1] = R / 2 - B / 2
    o[..., 2] = -R / 4 + G / 2 - B / 4
    return o


def ycocg_i16_to_rgb(y: np.ndarray) -> np.ndarray:
    """YCoCg.decode (:73-84): to_RGB in int16 (A4, wrapping), clip(0, 255), astype(uint8)."""
    Y, Co, Cg = (np.asarray(y, np.int64)[..., c] for c in range(3))
    o = np.stack([Y + Co - Cg, Y + Cg, Y - Co - Cg], axis=-1)
    o = ((o + 32768) % 65536 - 32768).astype(np.int16)
    return np.clip(o, 0, 255).astype(np.uint8)


def ycocg_dz_encode(rgb: np.ndarray, Q: int) -> np.ndarray:
    """YCoCg.encode (:33-56) with -a deadzone: int16 YCoCg, += [0,0,0], (x/Q).astype(int32) (A5), uint16."""
    x = ycocg_i16(rgb)
    return (x / Q).astype(np.int32).astype(np.uint16)


def ycocg_dz_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """YCoCg.decode (:58-85): astype(int16), Q * k in int16 (wrapping), -= 0, to_RGB, clip."""
    k16 = np.asarray(k, np.uint16).astype(np.int16).astype(np.int64)
    y = ((k16 * int(Q) + 32768) % 65536 - 32768).astype(np.int16)
    return ycocg_i16_to_rgb(y)


def ycocg_lm_encode(rgb: np.ndarray, Q: int, lo: int, hi: int):
    """YCoCg.encode with -a LloydMax: offset [-128, 0, 0] (:29-30) added to Y, LloydMax.quantize_fn,
    astype(uint16) -> (k, [centroids])."""
    x = ycocg_i16(rgb)
    x[..., 0] = (x[..., 0].astype(np.int32) - 128).astype(np.int16)
    k, cents = lm_quantize(x, Q, lo, hi)
    return k.astype(np.uint16), cents


def ycocg_lm_decode(k: np.ndarray, cents) -> np.ndarray:
    """YCoCg.decode with -a LloydMax: astype(int16), centroids into int16, Y + 128, to_RGB, clip."""
    y = lm_dequantize(np.asarray(k).astype(np.int16), cents)
    y[..., 0] = (y[..., 0].astype(np.int32) + 128).astype(np.int16)
    return ycocg_i16_to_rgb(y)


def dz_u8_encode(img: np.ndarray, Q: int) -> np.ndarray:
    """deadzone.encode (src/deadzone.py:67-79): astype(int16), (x/Q).astype(int32) (A5), astype(uint8)."""
    return (np.asarray(img).astype(np.int16) / Q).astype(np.int32).astype(np.uint8)


def dz_u8_decode(k: np.ndarray, Q: int) -> np.ndarray:
    """deadzone.decode (:81-93): Q * k with k uint8 and Q a Python int <= 255 -> uint8 (wrapping)."""
    return ((np.asarray(k, np.uint8).astype(np.int64) * int(Q)) & 0xFF).astype(np.uint8)
