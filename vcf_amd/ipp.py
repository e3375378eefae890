"""IPP temporal tools on the GPU (src/IPP_DCT.py): block matching, motion
compensation, residual and reconstruction through libvcf_amd.so.  Host
arrays in and out (the IPP driver keeps a GOP's frames on the device when it
calls the C ABI directly)."""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .device import DeviceBuffer


def _rgb(a):
    a = np.ascontiguousarray(a)
    if a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
        raise ValueError("expected H x W x 3 uint8")
    return a


def block_matching(ref: np.ndarray, cur: np.ndarray, bs: int = 16, sr: int = 8, fast: bool = False) -> np.ndarray:
    """IPP.block_matching (IPP_DCT.py:344-376) -> (H//bs, W//bs, 2) float32 (dx, dy)."""
    ref, cur = _rgb(ref), _rgb(cur)
    H, W = ref.shape[:2]
    mv = np.zeros((H // bs, W // bs, 2), np.float32)
    if mv.size == 0:
        return mv
    dr, dc = DeviceBuffer.from_array(ref), DeviceBuffer.from_array(cur)
    dm, dg = DeviceBuffer(mv.nbytes), DeviceBuffer(2 * H * W)
    try:
        L.call("vcf_ipp_block_match", dr.ptr, dc.ptr, H, W, int(bs), int(sr), int(bool(fast)), dm.ptr, dg.ptr, None)
        return dm.download(mv)
    finally:
        for b in (dr, dc, dm, dg):
            b.free()


def set_full_search_variant(variant: int) -> None:
    """0: word kernels (full search for bs % 4 == 0, parallel-round TSS for bs 16; default),
    1: byte / serial kernels (A/B; same vectors)."""
    L.call("vcf_ipp_set_full_search_variant", int(variant))


def motion_compensate(frame: np.ndarray, mv: np.ndarray, bs: int = 16) -> np.ndarray:
    frame = _rgb(frame)
    H, W = frame.shape[:2]
    mv = np.ascontiguousarray(mv, np.float32)
    if mv.shape != (H // bs, W // bs, 2):
        raise ValueError(f"motion field shape {mv.shape} != {(H // bs, W // bs, 2)}")
    out = np.empty_like(frame)
    df, dm, do = DeviceBuffer.from_array(frame), DeviceBuffer.from_array(mv if mv.size else np.zeros(2, np.float32)), \
        DeviceBuffer(frame.nbytes)
    try:
        L.call("vcf_ipp_motion_compensate", df.ptr, dm.ptr, H, W, int(bs), do.ptr, None)
        return do.download(out)
    finally:
        for b in (df, dm, do):
            b.free()


def _binary(name, a, b):
    a, b = np.ascontiguousarray(a, np.uint8), np.ascontiguousarray(b, np.uint8)
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    out = np.empty_like(a)
    if a.size == 0:
        return out
    da, db, do = DeviceBuffer.from_array(a), DeviceBuffer.from_array(b), DeviceBuffer(a.nbytes)
    try:
        L.call(name, da.ptr, db.ptr, a.size, do.ptr, None)
        return do.download(out)
    finally:
        for x in (da, db, do):
            x.free()


def residual(cur: np.ndarray, comp: np.ndarray) -> np.ndarray:
    """clip(cur - comp + 128, 0, 255) as uint8 (IPP_DCT.py:547-551)."""
    return _binary("vcf_ipp_residual", cur, comp)


def reconstruct(comp: np.ndarray, rec: np.ndarray) -> np.ndarray:
    """clip(comp + rec - 128, 0, 255) as uint8 (IPP_DCT.py:559-561)."""
    return _binary("vcf_ipp_reconstruct", comp, rec)


def rdo_modes(cur: np.ndarray, comp: np.ndarray, bs: int = 16, Q: int = 32, lam: float = 0.0,
              with_costs: bool = False):
    """-R block modes (IPP_DCT.py:441-468 + rdo_block_decision :290-342): (H//bs, W//bs) u8, 1 = I, 0 = P."""
    cur, comp = _rgb(cur), _rgb(comp)
    if cur.shape != comp.shape:
        raise ValueError("shape mismatch")
    H, W = cur.shape[:2]
    modes = np.zeros((H // bs, W // bs), np.uint8)
    costs = np.zeros((H // bs, W // bs, 4), np.float64)
    if modes.size == 0:
        return (modes, costs) if with_costs else modes
    dc, dp = DeviceBuffer.from_array(cur), DeviceBuffer.from_array(comp)
    dm, dk = DeviceBuffer(modes.nbytes), DeviceBuffer(costs.nbytes)
    try:
        L.call("vcf_ipp_rdo_modes", dc.ptr, dp.ptr, H, W, int(bs), int(Q), float(lam), dm.ptr, dk.ptr, None)
        dm.download(modes)
        dk.download(costs)
        return (modes, costs) if with_costs else modes
    finally:
        for b in (dc, dp, dm, dk):
            b.free()


def _modal(name, a, b, modes, bs):
    a, b = _rgb(a), _rgb(b)
    if a.shape != b.shape:
        raise ValueError("shape mismatch")
    H, W = a.shape[:2]
    m = np.ascontiguousarray(modes, np.uint8)
    if m.shape != (H // bs, W // bs):
        raise ValueError(f"mode map shape {m.shape} != {(H // bs, W // bs)}")
    out = np.empty_like(a)
    da, db, do = DeviceBuffer.from_array(a), DeviceBuffer.from_array(b), DeviceBuffer(a.nbytes)
    dm = DeviceBuffer.from_array(m if m.size else np.zeros(1, np.uint8))
    try:
        L.call(name, da.ptr, db.ptr, dm.ptr, H, W, int(bs), do.ptr, None)
        return do.download(out)
    finally:
        for x in (da, db, do, dm):
            x.free()


def rdo_residual(cur: np.ndarray, comp: np.ndarray, modes: np.ndarray, bs: int = 16) -> np.ndarray:
    """frame_to_encode_shifted (IPP_DCT.py:489-505)."""
    return _modal("vcf_ipp_rdo_residual", cur, comp, modes, bs)


def rdo_reconstruct(comp: np.ndarray, rec: np.ndarray, modes: np.ndarray, bs: int = 16) -> np.ndarray:
    """Mode-aware P-frame reconstruction (IPP_DCT.py:512-526, 770-790)."""
    return _modal("vcf_ipp_rdo_reconstruct", comp, rec, modes, bs)
