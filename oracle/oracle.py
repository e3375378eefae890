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
        srcs = [os.path.join(HERE, f) for f in ("vcf_oracle.c", "vcf_dwt_oracle.cpp", "vcf_ipp_oracle.c",
                                                       "vcf_dct_general_oracle.cpp")]
        if not os.path.exists(LIB_PATH) or any(os.path.getmtime(LIB_PATH) < os.path.getmtime(f) for f in srcs):
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
        # any block size (vcf_dct_general_oracle.cpp)
        L.vcfo_dct_supported.argtypes = [ctypes.c_int]
        L.vcfo_dct_uses_bluestein.argtypes = [ctypes.c_int]
        L.vcfo_cfft_f32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.vcfo_cfft_f64.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        for n in ("vcfo_dct2_f32_n", "vcfo_dct3_f32_n"):
            getattr(L, n).argtypes = [fp, ctypes.c_int, ctypes.c_int]
        for n in ("vcfo_dct2_f64_n", "vcfo_dct3_f64_n"):
            getattr(L, n).argtypes = [dp, ctypes.c_int, ctypes.c_int]
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.vcfo_dct_dz_encode_b.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_uint, u8p]
        L.vcfo_dct_dz_decode_b.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_uint, u8p]
        L.vcfo_dct_dz_encode_k32_b.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_uint, i32p]
        L.vcfo_ipp_rdo_modes.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_double, u8p, dp]
        L.vcfo_dct_dz_decode_k32_b.argtypes = [i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_uint, u8p]
        L.vcfo_dct_raw_encode_b.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint, fp]
        L.vcfo_dct_raw_decode_b.argtypes = [ctypes.POINTER(ctypes.c_int16), ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint, u8p]
        L.vcfo_perceptual_weights.argtypes = [dp]
        L.vcfo_dct_perceptual_tables.argtypes = [ctypes.c_int, u8p, u8p]
        # 2D-DWT path (vcf_dwt_oracle.cpp)
        ip = ctypes.POINTER(ctypes.c_int)
        u16p = ctypes.POINTER(ctypes.c_uint16)
        L.vcfo_wavelet_index.argtypes = [ctypes.c_char_p]
        L.vcfo_wavelet_len.argtypes = [ctypes.c_int]
        L.vcfo_dwt_shapes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ip]
        L.vcfo_dwt1_per_w.argtypes = [dp, ctypes.c_int, ctypes.c_int, dp, dp]
        L.vcfo_idwt1_per_w.argtypes = [dp, dp, ctypes.c_int, ctypes.c_int, dp]
        L.vcfo_wavedec2.argtypes = [dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp]
        L.vcfo_waverec2.argtypes = [dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp]
        L.vcfo_dwt_dz_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, u16p, u8p]
        L.vcfo_dwt_dz_decode.argtypes = [u16p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, u8p]
        # IPP temporal tools (vcf_ipp_oracle.c)
        L.vcfo_ipp_gray.argtypes = [u8p, ctypes.c_int64, u8p]
        L.vcfo_ipp_block_match.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, fp]
        L.vcfo_ipp_mc.argtypes = [u8p, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
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


def dct_supported(N: int) -> bool:
    return bool(lib().vcfo_dct_supported(int(N)))


def dct_uses_bluestein(N: int) -> bool:
    """pocketfft_r plans length N with Bluestein (fftblue over a cfftp of good_size_cmplx(2N-1))."""
    return bool(lib().vcfo_dct_uses_bluestein(int(N)))


def cfft(x, forward: bool = True):
    """pocketfft cfftp (scipy.fft.fft; backward unnormalised) along the last axis, complex64/128."""
    a = np.ascontiguousarray(x)
    assert a.dtype in (np.complex64, np.complex128)
    N = a.shape[-1]
    b = a.reshape(-1, N).copy()
    f = lib().vcfo_cfft_f32 if a.dtype == np.complex64 else lib().vcfo_cfft_f64
    if f(b.ctypes.data, N, b.shape[0], 1 if forward else 0) != 0:
        raise ValueError(f"length {N}: cfftp needs the generic passg (not restated)")
    return b.reshape(a.shape)


def dct_n(x, kind: int = 2, dtype=np.float32):
    """pocketfft DCT-II (kind 2) / DCT-III (kind 3), ortho, along the last axis, any supported length."""
    a = np.array(x, dtype=dtype)
    N = a.shape[-1]
    b = np.ascontiguousarray(a.reshape(-1, N))
    ct = ctypes.c_float if dtype == np.float32 else ctypes.c_double
    sfx = "f32" if dtype == np.float32 else "f64"
    f = getattr(lib(), f"vcfo_dct{kind}_{sfx}_n")
    if f(b.ctypes.data_as(ctypes.POINTER(ct)), N, b.shape[0]) != 0:
        raise ValueError(f"length {N} not covered by the restatement")
    return b.reshape(a.shape)


def perceptual_tables(B: int):
    """-p's JPEG tables resized to B x B (cv2.resize restated; unpinned for B != 8)."""
    y = np.empty((B, B), np.uint8)
    c = np.empty((B, B), np.uint8)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    if lib().vcfo_dct_perceptual_tables(int(B), y.ctypes.data_as(u8p), c.ctypes.data_as(u8p)) != 0:
        raise ValueError(B)
    return y, c


def encode_frame_b(rgb: np.ndarray, B: int, Q: int = 32, flags: int = 0, k32: bool = False) -> np.ndarray:
    """Any block size: u8 HxWx3 -> u8 HpxWpx3 (+128, wrapped) or, k32, the int32 k of the -L search."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    Hp, Wp = padded_shape(H, W, B)
    if k32:
        out = np.empty((Hp, Wp, 3), np.int32)
        rc = lib().vcfo_dct_dz_encode_k32_b(_u8(rgb), H, W, B, int(Q), flags,
                                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    else:
        out = np.empty((Hp, Wp, 3), np.uint8)
        rc = lib().vcfo_dct_dz_encode_b(_u8(rgb), H, W, B, int(Q), flags, _u8(out))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed ({rc})")
    return out


def decode_frame_b(k: np.ndarray, H: int, W: int, B: int, Q: int = 32, flags: int = 0) -> np.ndarray:
    """Any block size: u8 (decode_fn) or int32 (-L synthesis) HpxWpx3 -> u8 HxWx3."""
    Hp, Wp = padded_shape(H, W, B)
    if k.shape != (Hp, Wp, 3):
        raise ValueError(f"index array shape {k.shape} != {(Hp, Wp, 3)}")
    out = np.empty((H, W, 3), np.uint8)
    if k.dtype == np.int32:
        k = np.ascontiguousarray(k)
        rc = lib().vcfo_dct_dz_decode_k32_b(k.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), H, W, B, int(Q),
                                            flags, _u8(out))
    else:
        k = np.ascontiguousarray(k, dtype=np.uint8)
        rc = lib().vcfo_dct_dz_decode_b(_u8(k), H, W, B, int(Q), flags, _u8(out))
    if rc != 0:
        raise RuntimeError(f"oracle decode failed ({rc})")
    return out


def dct_raw_encode_b(rgb: np.ndarray, B: int, flags: int = 0) -> np.ndarray:
    """encode_fn with a quantizer other than deadzone (offset 0, 2D-DCT.py:106-109): the
    float32 HpxWpx3 coefficients (subband layout unless -x) handed to quantize_decom."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    Hp, Wp = padded_shape(H, W, B)
    out = np.empty((Hp, Wp, 3), np.float32)
    rc = lib().vcfo_dct_raw_encode_b(_u8(rgb), H, W, B, flags, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed ({rc})")
    return out


def dct_raw_decode_b(y: np.ndarray, H: int, W: int, B: int, flags: int = 0) -> np.ndarray:
    """decode_fn after another quantizer's dequantize_decom: int16 HpxWpx3 coefficients -> u8 HxWx3."""
    Hp, Wp = padded_shape(H, W, B)
    y = np.ascontiguousarray(y, dtype=np.int16)
    if y.shape != (Hp, Wp, 3):
        raise ValueError(f"coefficient array shape {y.shape} != {(Hp, Wp, 3)}")
    out = np.empty((H, W, 3), np.uint8)
    rc = lib().vcfo_dct_raw_decode_b(y.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), H, W, B, flags, _u8(out))
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


# --------------------------------------------------------------------------
# 2D-DWT path (src/2D-DWT.py encode_fn :57-78, decode_fn :80-101)
# --------------------------------------------------------------------------
def wavelet_index(name: str) -> int:
    i = lib().vcfo_wavelet_index(name.encode())
    if i < 0:
        raise ValueError(f"unknown wavelet {name!r}")
    return i


def dwt_shapes(H: int, W: int, levels: int):
    """[(h_l, w_l) for l = 1..levels] (mode 'per': ceil halving)."""
    hs = (ctypes.c_int * levels)()
    ws = (ctypes.c_int * levels)()
    lib().vcfo_dwt_shapes(H, W, levels, hs, ws)
    return list(zip(hs[:], ws[:]))


def subband_names(levels: int):
    """File order of write_decom_fn (2D-DWT.py:162-200)."""
    return [f"LL_{levels}"] + [f"{s}_{r}" for r in range(levels, 0, -1) for s in ("LH", "HL", "HH")]


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _coeff_count(H, W, levels):
    sh = dwt_shapes(H, W, levels)
    return sh[-1][0] * sh[-1][1] + sum(3 * h * w for h, w in sh)


def dwt1(x: np.ndarray, wavelet: str):
    """pywt.dwt(x, wavelet, mode='periodization') of one float64 line."""
    x = np.ascontiguousarray(x, np.float64)
    n = (x.size + 1) // 2
    cA, cD = np.empty(n), np.empty(n)
    dp = ctypes.POINTER(ctypes.c_double)
    if lib().vcfo_dwt1_per_w(x.ctypes.data_as(dp), x.size, wavelet_index(wavelet), cA.ctypes.data_as(dp),
                             cD.ctypes.data_as(dp)) != 0:
        raise ValueError(wavelet)
    return cA, cD


def idwt1(a: np.ndarray, d: np.ndarray, wavelet: str):
    """pywt.idwt(a, d, wavelet, mode='periodization') of one pair of float64 lines."""
    a = np.ascontiguousarray(a, np.float64)
    d = np.ascontiguousarray(d, np.float64)
    out = np.empty(2 * a.size)
    dp = ctypes.POINTER(ctypes.c_double)
    if lib().vcfo_idwt1_per_w(a.ctypes.data_as(dp), d.ctypes.data_as(dp), a.size, wavelet_index(wavelet),
                              out.ctypes.data_as(dp)) != 0:
        raise ValueError(wavelet)
    return out


def wavedec2(x: np.ndarray, wavelet: str, levels: int):
    """pywt.wavedec2(x, wavelet, mode='per', level=levels) as [cA, (cH, cV, cD), ...]."""
    x = np.ascontiguousarray(x, np.float64)
    H, W = x.shape
    flat = np.empty(_coeff_count(H, W, levels))
    rc = lib().vcfo_wavedec2(_dp(x), H, W, wavelet_index(wavelet), levels, _dp(flat))
    if rc != 0:
        raise RuntimeError("oracle wavedec2 failed")
    sh = dwt_shapes(H, W, levels)
    h, w = sh[-1]
    out = [flat[:h * w].reshape(h, w)]
    off = h * w
    for r in range(levels, 0, -1):
        h, w = sh[r - 1]
        out.append(tuple(flat[off + k * h * w:off + (k + 1) * h * w].reshape(h, w) for k in range(3)))
        off += 3 * h * w
    return out


def waverec2(coeffs, wavelet: str, H: int, W: int):
    """pywt.waverec2(coeffs, wavelet, mode='per') for a plane of H x W."""
    levels = len(coeffs) - 1
    flat = np.concatenate([np.ravel(coeffs[0])] + [np.ravel(b) for r in coeffs[1:] for b in r]).astype(np.float64)
    sh = dwt_shapes(H, W, levels)
    out = np.empty((2 * sh[0][0], 2 * sh[0][1]))
    rc = lib().vcfo_waverec2(_dp(flat), H, W, wavelet_index(wavelet), levels, _dp(out))
    if rc != 0:
        raise RuntimeError("oracle waverec2 failed")
    return out


def dwt_encode_frame(rgb: np.ndarray, wavelet: str = "db5", levels: int = 5, Q: int = 32):
    """u8 RGB -> {subband name: u16 (LL) / u8 (details) H_l x W_l x 3}."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    H, W = rgb.shape[:2]
    sh = dwt_shapes(H, W, levels)
    LL = np.empty((sh[-1][0], sh[-1][1], 3), np.uint16)
    det = np.empty(3 * sum(3 * h * w for h, w in sh), np.uint8)
    rc = lib().vcfo_dwt_dz_encode(_u8(rgb), H, W, wavelet_index(wavelet), levels, int(Q),
                                  LL.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), _u8(det))
    if rc != 0:
        raise RuntimeError("oracle dwt encode failed")
    out = {f"LL_{levels}": LL}
    off = 0
    for r in range(levels, 0, -1):
        h, w = sh[r - 1]
        for s in ("LH", "HL", "HH"):
            out[f"{s}_{r}"] = det[off:off + 3 * h * w].reshape(h, w, 3)
            off += 3 * h * w
    return out


def dwt_decode_frame(subbands, H: int, W: int, wavelet: str = "db5", levels: int = 5, Q: int = 32):
    """{subband: indices} -> u8 RGB (2*ceil(H/2) x 2*ceil(W/2) x 3, like pywt.waverec2)."""
    sh = dwt_shapes(H, W, levels)
    LL = np.ascontiguousarray(subbands[f"LL_{levels}"], np.uint16)
    det = np.concatenate([np.ravel(np.ascontiguousarray(subbands[f"{s}_{r}"], np.uint8))
                          for r in range(levels, 0, -1) for s in ("LH", "HL", "HH")])
    out = np.empty((2 * sh[0][0], 2 * sh[0][1], 3), np.uint8)
    rc = lib().vcfo_dwt_dz_decode(LL.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), _u8(det), H, W,
                                  wavelet_index(wavelet), levels, int(Q), _u8(out))
    if rc != 0:
        raise RuntimeError("oracle dwt decode failed")
    return out


# ---- IPP (src/IPP_DCT.py; vcf_ipp_oracle.c) ----

def ipp_gray(rgb: np.ndarray) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.uint8)
    out = np.empty(rgb.shape[:2], np.uint8)
    lib().vcfo_ipp_gray(_u8(rgb), rgb.shape[0] * rgb.shape[1], _u8(out))
    return out


def ipp_block_matching(ref, cur, bs=16, sr=8, fast=False) -> np.ndarray:
    ref, cur = np.ascontiguousarray(ref, np.uint8), np.ascontiguousarray(cur, np.uint8)
    H, W = ref.shape[:2]
    mv = np.zeros((H // bs, W // bs, 2), np.float32)
    lib().vcfo_ipp_block_match(_u8(ref), _u8(cur), H, W, bs, sr, int(bool(fast)),
                               mv.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return mv


def ipp_motion_compensate(frame, mv, bs=16) -> np.ndarray:
    frame = np.ascontiguousarray(frame, np.uint8)
    mv = np.ascontiguousarray(mv, np.float32)
    out = np.empty_like(frame)
    H, W = frame.shape[:2]
    lib().vcfo_ipp_mc(_u8(frame), mv.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), H, W, bs, _u8(out))
    return out


def ipp_rdo_modes(cur, comp, bs=16, qss=32, lam=1.0, with_costs=False):
    """IPP -R block modes (1 = I, 0 = P) of cur against its compensation comp."""
    cur, comp = np.ascontiguousarray(cur, np.uint8), np.ascontiguousarray(comp, np.uint8)
    H, W = cur.shape[:2]
    modes = np.zeros((H // bs, W // bs), np.uint8)
    costs = np.zeros((H // bs, W // bs, 4), np.float64)
    rc = lib().vcfo_ipp_rdo_modes(_u8(cur), _u8(comp), H, W, bs, int(qss), float(lam), _u8(modes),
                                  costs.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc != 0:
        raise RuntimeError(f"oracle rdo failed ({rc})")
    return (modes, costs) if with_costs else modes


def ipp_rdo_residual(cur, comp, modes, bs=16):
    """:489-505: P blocks clip(cur - comp + 128), I blocks cur, outside full blocks 128."""
    H, W = cur.shape[:2]
    out = np.full_like(cur, 128)
    for by in range(H // bs):
        for bx in range(W // bs):
            sl = (slice(by * bs, (by + 1) * bs), slice(bx * bs, (bx + 1) * bs))
            c = cur[sl].astype(np.int32)
            out[sl] = c if modes[by, bx] else np.clip(c - comp[sl].astype(np.int32) + 128, 0, 255)
    return out


def ipp_rdo_reconstruct(comp, rec, modes, bs=16):
    """:512-526: P blocks clip(comp + rec - 128), I blocks rec, outside full blocks 0."""
    H, W = comp.shape[:2]
    out = np.zeros_like(comp)
    for by in range(H // bs):
        for bx in range(W // bs):
            sl = (slice(by * bs, (by + 1) * bs), slice(bx * bs, (bx + 1) * bs))
            r = rec[sl].astype(np.int32)
            out[sl] = r if modes[by, bx] else np.clip(comp[sl].astype(np.int32) + r - 128, 0, 255)
    return out


def ipp_residual(cur, comp) -> np.ndarray:
    """IPP_DCT.py:547-551."""
    return np.clip(cur.astype(np.int16) - comp.astype(np.int16) + 128, 0, 255).astype(np.uint8)


def ipp_reconstruct(comp, rec) -> np.ndarray:
    """IPP_DCT.py:559-561."""
    return np.clip(comp.astype(np.int16) + rec.astype(np.int16) - 128, 0, 255).astype(np.uint8)
