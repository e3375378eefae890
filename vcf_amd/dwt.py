"""2D-DWT + deadzone on the GPU (src/2D-DWT.py encode_fn :57-78 up to the
TIFF writer, decode_fn :80-101 after the TIFF reader), through
libvcf_amd.so (vcf_dwt_dz_encode / vcf_dwt_dz_decode).  No CPU path.

lifting=True selects the opt-in lifting form of bior4.4 (vcf_dwt_dz_*_lift,
csrc/vcf_dwt_lift.h): not bit-exact -- indices and decoded bytes within +-1
of the default path (the lifting form)."""
from __future__ import annotations

import ctypes
import functools

import numpy as np

from . import _lib as L
from .device import DeviceBuffer


def wavelet_index(name: str) -> int:
    i = ctypes.c_int32()
    L.call("vcf_wavelet_index", str(name).encode(), ctypes.byref(i))
    return i.value


@functools.lru_cache(maxsize=64)
def layout(H: int, W: int, levels: int):
    """([(h_l, w_l) for l = 1..levels], packed bytes per frame, workspace bytes per frame)."""
    hs = (ctypes.c_int32 * levels)()
    ws = (ctypes.c_int32 * levels)()
    pb, wb = ctypes.c_int64(), ctypes.c_int64()
    L.call("vcf_dwt_layout", H, W, levels, hs, ws, ctypes.byref(pb), ctypes.byref(wb))
    return list(zip(hs[:], ws[:])), pb.value, wb.value


def subband_names(levels: int):
    """File order of write_decom_fn (2D-DWT.py:162-200)."""
    return [f"LL_{levels}"] + [f"{s}_{r}" for r in range(levels, 0, -1) for s in ("LH", "HL", "HH")]


def unpack(packed: np.ndarray, H: int, W: int, levels: int):
    """Packed bytes of one frame -> {name: u16 LL / u8 detail array (h x w x 3)}."""
    shapes, _, _ = layout(H, W, levels)
    h, w = shapes[-1]
    out = {f"LL_{levels}": packed[:h * w * 6].view(np.uint16).reshape(h, w, 3)}
    off = h * w * 6
    for r in range(levels, 0, -1):
        h, w = shapes[r - 1]
        for s in ("LH", "HL", "HH"):
            out[f"{s}_{r}"] = packed[off:off + h * w * 3].reshape(h, w, 3)
            off += h * w * 3
    return out


def pack(subbands, H: int, W: int, levels: int) -> np.ndarray:
    parts = [np.ascontiguousarray(subbands[f"LL_{levels}"], np.uint16).view(np.uint8).ravel()]
    for r in range(levels, 0, -1):
        for s in ("LH", "HL", "HH"):
            parts.append(np.ascontiguousarray(subbands[f"{s}_{r}"], np.uint8).ravel())
    return np.concatenate(parts)


def _frames(a, what):
    a = np.asarray(a)
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4 or a.shape[-1] != 3 or a.dtype != np.uint8:
        raise ValueError(f"{what}: expected (N,) H x W x 3 uint8")
    return np.ascontiguousarray(a)


def _entry(name: str, lifting: bool) -> str:
    return name + "_lift" if lifting else name


def encode_device(din: DeviceBuffer, n: int, H: int, W: int, wavelet: int, levels: int, Q: int,
                  packed: DeviceBuffer, workspace: DeviceBuffer, stream=None, lifting: bool = False) -> None:
    """n HBM-resident H x W x 3 u8 frames -> their packed subbands (layout()'s
    bytes per frame), enqueued on `stream`; `wavelet` is wavelet_index()'s."""
    _, pb, wb = layout(H, W, levels)
    if din.nbytes < n * H * W * 3 or packed.nbytes < n * pb or workspace.nbytes < n * wb:
        raise ValueError("dwt encode_device: buffer smaller than n frames need")
    L.call(_entry("vcf_dwt_dz_encode", lifting), din.ptr, n, H, W, int(wavelet), levels, int(Q), packed.ptr,
           workspace.ptr, None if stream is None else stream.handle)


def decode_device(packed: DeviceBuffer, n: int, H: int, W: int, wavelet: int, levels: int, Q: int,
                  out: DeviceBuffer, workspace: DeviceBuffer, stream=None, lifting: bool = False) -> None:
    """n frames' packed subbands in HBM -> u8 RGB (2*ceil(H/2) x 2*ceil(W/2) x 3 each)."""
    shapes, pb, wb = layout(H, W, levels)
    if packed.nbytes < n * pb or out.nbytes < n * 4 * shapes[0][0] * shapes[0][1] * 3 or workspace.nbytes < n * wb:
        raise ValueError("dwt decode_device: buffer smaller than n frames need")
    L.call(_entry("vcf_dwt_dz_decode", lifting), packed.ptr, n, H, W, int(wavelet), levels, int(Q), out.ptr,
           workspace.ptr, None if stream is None else stream.handle)


def encode(rgb: np.ndarray, wavelet: str = "db5", levels: int = 5, Q: int = 32, variant: int = 0,
           lifting: bool = False):
    """HxWx3 u8 (or N of them) -> list of {subband name: indices} per frame.
    variant: 0 the product kernels; any other value a variant of the A/B library
    (include/vcf_amd_ab.h: 1 fused level kernels, 2 separable kernels, 6 strip kernels on every
    level, ...; A/B records and cross-checks, not the product path)."""
    f = _frames(rgb, "rgb")
    n, H, W, _ = f.shape
    _, pb, wb = layout(H, W, levels)
    din, dout, dws = DeviceBuffer.from_array(f), DeviceBuffer(n * pb), DeviceBuffer(n * wb)
    try:
        if variant and lifting:
            raise ValueError("lifting is a product entry point, not an A/B variant")
        if variant == 0:
            L.call(_entry("vcf_dwt_dz_encode", lifting), din.ptr, n, H, W, wavelet_index(wavelet), levels, int(Q),
                   dout.ptr, dws.ptr, None)
        else:
            L.call_ab("vcf_dwt_dz_encode_variant", int(variant), din.ptr, n, H, W, wavelet_index(wavelet), levels,
                      int(Q), dout.ptr, dws.ptr, None)
        packed = dout.download(np.empty((n, pb), np.uint8))
    finally:
        din.free()
        dout.free()
        dws.free()
    return [unpack(packed[i], H, W, levels) for i in range(n)]


def decode(subbands, H: int, W: int, wavelet: str = "db5", levels: int = 5, Q: int = 32,
           variant: int = 0, lifting: bool = False) -> np.ndarray:
    """{name: indices} (or a list of them) -> u8 RGB (2*ceil(H/2) x 2*ceil(W/2) x 3 each)."""
    single = isinstance(subbands, dict)
    sets = [subbands] if single else list(subbands)
    shapes, pb, wb = layout(H, W, levels)
    packed = np.stack([pack(s, H, W, levels) for s in sets])
    n = len(sets)
    Ho, Wo = 2 * shapes[0][0], 2 * shapes[0][1]
    din, dout, dws = DeviceBuffer.from_array(packed), DeviceBuffer(n * Ho * Wo * 3), DeviceBuffer(n * wb)
    try:
        if variant and lifting:
            raise ValueError("lifting is a product entry point, not an A/B variant")
        if variant == 0:
            L.call(_entry("vcf_dwt_dz_decode", lifting), din.ptr, n, H, W, wavelet_index(wavelet), levels, int(Q),
                   dout.ptr, dws.ptr, None)
        else:
            L.call_ab("vcf_dwt_dz_decode_variant", int(variant), din.ptr, n, H, W, wavelet_index(wavelet), levels,
                      int(Q), dout.ptr, dws.ptr, None)
        out = dout.download(np.empty((n, Ho, Wo, 3), np.uint8))
    finally:
        din.free()
        dout.free()
        dws.free()
    return out[0] if single else out


def lift_coefficients(rgb: np.ndarray, levels: int = 5):
    """The opt-in lifting path's float64 coefficients of one HxWx3 u8 frame
    before quantization (vcf_dwt_lift_analyze_f64, bior4.4): [cA, (cH, cV, cD)
    per level, coarsest first] per YCoCg channel, pywt.wavedec2's order and
    naming (cH = the reference's LH, cV = HL, cD = HH)."""
    f = _frames(rgb, "rgb")
    if f.shape[0] != 1:
        raise ValueError("one frame")
    _, H, W, _ = f.shape
    shapes, pb, wb = layout(H, W, levels)
    n_coef = sum(9 * h * w for h, w in shapes) + 3 * shapes[-1][0] * shapes[-1][1]
    din, dco, dpk, dws = DeviceBuffer.from_array(f), DeviceBuffer(8 * n_coef), DeviceBuffer(pb), DeviceBuffer(wb)
    try:
        L.call("vcf_dwt_lift_analyze_f64", din.ptr, H, W, levels, dco.ptr, dpk.ptr, dws.ptr, None)
        flat = dco.download(np.empty(n_coef, np.float64))
    finally:
        for b in (din, dco, dpk, dws):
            b.free()
    det, off = [], 0
    for h, w in shapes:
        d = flat[off:off + 9 * h * w].reshape(3, 3, h, w)   # [LH, HL, HH][channel]
        det.append(d)
        off += 9 * h * w
    h, w = shapes[-1]
    ll = flat[off:off + 3 * h * w].reshape(3, h, w)
    return [[ll[c]] + [tuple(det[lv][s, c] for s in range(3)) for lv in range(levels - 1, -1, -1)]
            for c in range(3)]
