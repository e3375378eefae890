"""ctypes front-end of the CPU oracle (oracle/vcf_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker, never as the product.
The product path (vcf_amd/) never imports this module.

Restates src/2D-DCT.py:268-372 (encode_fn up to the entropy codec) and
src/2D-DCT.py:377-466 (decode_fn after the entropy decoder) of the reference,
with the upstream-package assumptions A1-A5 of SURVEY.md Appendix A.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

FLAG_NO_SUBBANDS = 1   # -x  (2D-DCT.py:40)
FLAG_PERCEPTUAL = 2    # -p  (2D-DCT.py:38)

_lib = None


def build() -> str:
    """Compile the oracle (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "vcf_oracle.c"))
        ):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.vcfo_dct_dz_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint, u8p]
        L.vcfo_dct_dz_decode.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint, u8p]
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        for n in ("vcfo_dct2_8_f32", "vcfo_dct3_8_f32"):
            getattr(L, n).argtypes = [fp]
        for n in ("vcfo_dct2_8_f64", "vcfo_dct3_8_f64"):
            getattr(L, n).argtypes = [dp]
        L.vcfo_pocketfft_consts.argtypes = [fp, dp, fp, dp, fp, dp]
        L.vcfo_perceptual_weights.argtypes = [dp]
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def padded_shape(H: int, W: int, B: int = 8):
    """2D-DCT.py:208-209: next multiple of the block size."""
    return (H + B - 1) // B * B, (W + B - 1) // B * B


def encode_frame(rgb: np.ndarray, Q: int = 32, flags: int = 0) -> np.ndarray:
    """u8 HxWx3 RGB -> u8 HpxWpx3 deadzone indices (+128, subband layout)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    if rgb.ndim != 3 or rgb.shape[2] != 3:
        raise ValueError("Input image must be a 3D array (height, width, channels).")
    H, W = rgb.shape[:2]
    Hp, Wp = padded_shape(H, W)
    out = np.empty((Hp, Wp, 3), np.uint8)
    rc = lib().vcfo_dct_dz_encode(_u8(rgb), H, W, int(Q), flags, _u8(out))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed ({rc})")
    return out


def decode_frame(k: np.ndarray, H: int, W: int, Q: int = 32, flags: int = 0) -> np.ndarray:
    """u8 HpxWpx3 indices -> u8 HxWx3 reconstruction."""
    k = np.ascontiguousarray(k, dtype=np.uint8)
    Hp, Wp = padded_shape(H, W)
    if k.shape != (Hp, Wp, 3):
        raise ValueError(f"index array shape {k.shape} != {(Hp, Wp, 3)}")
    out = np.empty((H, W, 3), np.uint8)
    rc = lib().vcfo_dct_dz_decode(_u8(k), H, W, int(Q), flags, _u8(out))
    if rc != 0:
        raise RuntimeError(f"oracle decode failed ({rc})")
    return out


def _vec8(fn, x, dtype):
    a = np.array(x, dtype=dtype).reshape(-1, 8).copy()
    ct = ctypes.c_float if dtype == np.float32 else ctypes.c_double
    for row in a:
        fn(row.ctypes.data_as(ctypes.POINTER(ct)))
    return a


def dct2_8(x, dtype=np.float32):
    """pocketfft DCT-II, N=8, ortho, on each row of x (shape [..., 8])."""
    f = lib().vcfo_dct2_8_f32 if dtype == np.float32 else lib().vcfo_dct2_8_f64
    return _vec8(f, x, dtype).reshape(np.shape(x))


def dct3_8(x, dtype=np.float64):
    """pocketfft DCT-III (= idct type 2), N=8, ortho, on each row of x."""
    f = lib().vcfo_dct3_8_f32 if dtype == np.float32 else lib().vcfo_dct3_8_f64
    return _vec8(f, x, dtype).reshape(np.shape(x))


def pocketfft_consts():
    twf = (ctypes.c_float * 8)()
    twd = (ctypes.c_double * 8)()
    rf = (ctypes.c_float * 2)()
    rd = (ctypes.c_double * 2)()
    s2f = ctypes.c_float()
    s2d = ctypes.c_double()
    lib().vcfo_pocketfft_consts(twf, twd, rf, rd, ctypes.byref(s2f), ctypes.byref(s2d))
    return dict(tw_f32=np.array(twf[:], np.float32), tw_f64=np.array(twd[:]),
                rfft_f32=np.array(rf[:], np.float32), rfft_f64=np.array(rd[:]),
                sqrt2_f32=np.float32(s2f.value), sqrt2_f64=s2d.value)


def perceptual_weights() -> np.ndarray:
    w = np.empty((3, 8, 8), np.float64)
    lib().vcfo_perceptual_weights(w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return w


# --------------------------------------------------------------------------
# Reference-faithful numpy restatement used as the "port" CPU baseline in
# bench.py: the same per-block structure as the reference (scipy-free, one
# call per 8x8 block and channel would take minutes; this vectorizes over
# blocks with the oracle's exact C transform instead).
# --------------------------------------------------------------------------
def encode_frames(frames: np.ndarray, Q: int = 32, flags: int = 0) -> np.ndarray:
    return np.stack([encode_frame(f, Q, flags) for f in frames])
