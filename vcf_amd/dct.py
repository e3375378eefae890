"""DCT + deadzone hot path on the GPU (include/vcf_amd.h vcf_dct_dz_*).

Replaces, in one fused kernel per direction, the numpy/scipy span of
src/2D-DCT.py encode_fn :276-361 (to the uint8 indices handed to the entropy
codec) and decode_fn :399-466 (from the entropy decoder's uint8 array to the
clipped RGB frame).  B = 8 runs the fused 8x8 kernels; the other -B sizes
(block_size_supported) the generic-B kernels.  encode_k32/decode_k32 are the
int32 analysis/synthesis of the -L search (optimize_block_size :533-579).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import VCF_DCT_NO_SUBBANDS, VCF_DCT_PERCEPTUAL, call, call_ab
from .device import DeviceBuffer, _h

__all__ = ["padded_shape", "flags_from", "encode_device", "decode_device", "encode", "decode",
           "block_size_supported", "encode_k32", "decode_k32", "raw_encode_device", "raw_decode_device",
           "VCF_DCT_NO_SUBBANDS", "VCF_DCT_PERCEPTUAL"]


def block_size_supported(block_size: int) -> bool:
    """True if the HIP path has a transform of this length: any 1 <= B <= 4096 (compiled
    kernels for the 5-smooth B <= 128, run-time plans otherwise -- rfftp, or Bluestein for
    the lengths pocketfft plans that way, 191, 199, ...)."""
    return bool(_lib.lib().vcf_dct_block_size_supported(int(block_size)))


def padded_shape(H: int, W: int, block_size: int = 8):
    hp, wp = ctypes.c_int32(), ctypes.c_int32()
    call("vcf_dct_padded_shape", H, W, block_size, ctypes.byref(hp), ctypes.byref(wp))
    return hp.value, wp.value


def flags_from(disable_subbands: bool = False, perceptual: bool = False) -> int:
    return (VCF_DCT_NO_SUBBANDS if disable_subbands else 0) | (VCF_DCT_PERCEPTUAL if perceptual else 0)


def encode_device(rgb: DeviceBuffer, n_frames: int, H: int, W: int, Q: int = 32, flags: int = 0,
                  out: DeviceBuffer | None = None, stream=None, block_size: int = 8,
                  variant: int = 0) -> DeviceBuffer:
    """Frames resident in HBM -> coefficient frames in HBM (asynchronous on `stream`).

    variant: 0 the product kernels, -1 the generic-B kernels (any supported B, 8 included), any
    other value a kernel variant of the A/B library (include/vcf_amd_ab.h: A/B records and
    cross-checks, not the product path)."""
    Hp, Wp = padded_shape(H, W, block_size)
    if rgb.nbytes < n_frames * H * W * 3:
        raise ValueError("input buffer too small")
    if out is None:
        out = DeviceBuffer(n_frames * Hp * Wp * 3)
    elif out.nbytes < n_frames * Hp * Wp * 3:
        raise ValueError("output buffer too small")
    if variant == -1:
        call("vcf_dct_dz_encode_any", rgb.ptr, n_frames, H, W, block_size, int(Q), flags, out.ptr, _h(stream))
    elif variant == 0:
        call("vcf_dct_dz_encode", rgb.ptr, n_frames, H, W, block_size, int(Q), flags, out.ptr, _h(stream))
    else:
        call_ab("vcf_dct_dz_encode_variant", variant, rgb.ptr, n_frames, H, W, block_size, int(Q), flags,
                out.ptr, _h(stream))
    return out


def decode_device(k: DeviceBuffer, n_frames: int, H: int, W: int, Q: int = 32, flags: int = 0,
                  out: DeviceBuffer | None = None, stream=None, block_size: int = 8,
                  variant: int = 0) -> DeviceBuffer:
    """variant: 0 the product kernels, -1 the generic-B kernels (any supported B, 8 included),
    any other value a decode variant of the A/B library (include/vcf_amd_ab.h)."""
    Hp, Wp = padded_shape(H, W, block_size)
    if k.nbytes < n_frames * Hp * Wp * 3:
        raise ValueError("input buffer too small")
    if out is None:
        out = DeviceBuffer(n_frames * H * W * 3)
    elif out.nbytes < n_frames * H * W * 3:
        raise ValueError("output buffer too small")
    if variant == -1:
        call("vcf_dct_dz_decode_any", k.ptr, n_frames, H, W, block_size, int(Q), flags, out.ptr, _h(stream))
    elif variant == 0:
        call("vcf_dct_dz_decode", k.ptr, n_frames, H, W, block_size, int(Q), flags, out.ptr, _h(stream))
    else:
        call_ab("vcf_dct_dz_decode_variant", variant, k.ptr, n_frames, H, W, block_size, int(Q), flags,
                out.ptr, _h(stream))
    return out


def _frames(a: np.ndarray, what: str) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype != np.uint8:
        raise TypeError(f"{what} must be uint8, got {a.dtype}")
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4 or a.shape[3] != 3:
        raise ValueError("Input image must be a 3D array (height, width, channels).")
    return np.ascontiguousarray(a)


def encode(rgb: np.ndarray, Q: int = 32, flags: int = 0, block_size: int = 8,
           variant: int = 0) -> np.ndarray:
    """Host convenience: HxWx3 (or NxHxWx3) u8 -> HpxWpx3 (NxHpxWpx3) u8 indices."""
    single = np.asarray(rgb).ndim == 3
    f = _frames(rgb, "rgb")
    n, H, W, _ = f.shape
    Hp, Wp = padded_shape(H, W, block_size)
    din = DeviceBuffer.from_array(f)
    dout = encode_device(din, n, H, W, Q, flags, block_size=block_size, variant=variant)
    res = dout.download(np.empty((n, Hp, Wp, 3), np.uint8))
    din.free()
    dout.free()
    return res[0] if single else res


def decode(k: np.ndarray, H: int, W: int, Q: int = 32, flags: int = 0, block_size: int = 8,
           variant: int = 0) -> np.ndarray:
    """Host convenience: HpxWpx3 (or N...) u8 indices -> HxWx3 u8 reconstruction."""
    single = np.asarray(k).ndim == 3
    f = _frames(k, "k")
    n = f.shape[0]
    Hp, Wp = padded_shape(H, W, block_size)
    if f.shape[1:3] != (Hp, Wp):
        raise ValueError(f"index frames {f.shape[1:3]} do not match {(Hp, Wp)} for {H}x{W}")
    din = DeviceBuffer.from_array(f)
    dout = decode_device(din, n, H, W, Q, flags, block_size=block_size, variant=variant)
    res = dout.download(np.empty((n, H, W, 3), np.uint8))
    din.free()
    dout.free()
    return res[0] if single else res


def encode_k32(rgb: np.ndarray, Q: int = 32, flags: int = 0, block_size: int = 8) -> np.ndarray:
    """-L analysis (2D-DCT.py:538-545): HxWx3 (or N...) u8 -> HpxWpx3 int32 k, before +128/uint8."""
    single = np.asarray(rgb).ndim == 3
    f = _frames(rgb, "rgb")
    n, H, W, _ = f.shape
    Hp, Wp = padded_shape(H, W, block_size)
    din = DeviceBuffer.from_array(f)
    dout = DeviceBuffer(n * Hp * Wp * 3 * 4)
    call("vcf_dct_dz_encode_k32", din.ptr, n, H, W, block_size, int(Q), flags, dout.ptr, None)
    res = dout.download(np.empty((n, Hp, Wp, 3), np.int32))
    din.free()
    dout.free()
    return res[0] if single else res


def decode_k32(k: np.ndarray, H: int, W: int, Q: int = 32, flags: int = 0, block_size: int = 8) -> np.ndarray:
    """-L synthesis (2D-DCT.py:560-568): HpxWpx3 (or N...) int32 k -> HxWx3 u8."""
    k = np.asarray(k)
    if k.dtype != np.int32:
        raise TypeError(f"k must be int32, got {k.dtype}")
    single = k.ndim == 3
    f = np.ascontiguousarray(k[None] if single else k)
    n = f.shape[0]
    Hp, Wp = padded_shape(H, W, block_size)
    if f.shape[1:] != (Hp, Wp, 3):
        raise ValueError(f"index frames {f.shape[1:]} do not match {(Hp, Wp, 3)} for {H}x{W}")
    din = DeviceBuffer.from_array(f)
    dout = DeviceBuffer(n * H * W * 3)
    call("vcf_dct_dz_decode_k32", din.ptr, n, H, W, block_size, int(Q), flags, dout.ptr, None)
    res = dout.download(np.empty((n, H, W, 3), np.uint8))
    din.free()
    dout.free()
    return res[0] if single else res


def raw_encode_device(rgb: DeviceBuffer, n_frames: int, H: int, W: int, flags: int = 0,
                      out: DeviceBuffer | None = None, stream=None, block_size: int = 8) -> DeviceBuffer:
    """encode_fn up to the quantizer for -a other than deadzone (offset 0, 2D-DCT.py:106-109):
    u8 RGB frames -> float32 HpxWpx3 coefficient frames (subband layout unless -x, -p applied)."""
    Hp, Wp = padded_shape(H, W, block_size)
    if rgb.nbytes < n_frames * H * W * 3:
        raise ValueError("input buffer too small")
    if out is None:
        out = DeviceBuffer(n_frames * Hp * Wp * 3 * 4)
    elif out.nbytes < n_frames * Hp * Wp * 3 * 4:
        raise ValueError("output buffer too small")
    call("vcf_dct_raw_encode", rgb.ptr, n_frames, H, W, block_size, flags, out.ptr, _h(stream))
    return out


def raw_decode_device(coef: DeviceBuffer, n_frames: int, H: int, W: int, flags: int = 0,
                      out: DeviceBuffer | None = None, stream=None, block_size: int = 8) -> DeviceBuffer:
    """decode_fn after another quantizer's dequantize_decom: int16 HpxWpx3 coefficient frames -> u8 RGB."""
    Hp, Wp = padded_shape(H, W, block_size)
    if coef.nbytes < n_frames * Hp * Wp * 3 * 2:
        raise ValueError("input buffer too small")
    if out is None:
        out = DeviceBuffer(n_frames * H * W * 3)
    elif out.nbytes < n_frames * H * W * 3:
        raise ValueError("output buffer too small")
    call("vcf_dct_raw_decode", coef.ptr, n_frames, H, W, block_size, flags, out.ptr, _h(stream))
    return out
