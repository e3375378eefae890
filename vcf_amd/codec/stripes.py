"""One large frame sharded by block-row stripes across the ranks (SURVEY.md §8(e),
"Single large frame": DCT + deadzone, row stripes, gather).

The B x B DCT + deadzone of src/2D-DCT.py encode_fn :276-361 / decode_fn
:399-466 has no halo: every block is coded from its own B x B pixels, and the
color transform, offset, -p weights and the quantizer are per pixel or per
coefficient.  The only frame-wide steps are

- the centred zero padding (pad_and_center_to_multiple_of_block_size
  :191-229, zero RGB pixels added before the offset), and
- the subband reordering (get_subbands, :330-345): coefficient (i, j) of
  block (by, bx) goes to row i * nby + by, column j * nbx + bx.

So rank r takes the block rows [by0, by1) = frame_range(nby, r, P) of the
padded frame: it builds that stripe of the padded frame (its own image rows
plus the zero rows of the top/bottom padding that fall in it, width W, the
horizontal padding left to the kernel, which centres it the same way),
codes it as a B*(by1-by0) x W frame -- a stripe is a multiple of B tall, so
the kernel adds no vertical padding -- and rank 0 scatters the gathered
stripes' rows i * nbs + b to the frame's rows i * nby + by0 + b (with -x,
no reordering, a stripe is a contiguous slab).  Decoding is the inverse:
every rank picks its stripe's rows out of the frame's indices, decodes them
to B*(by1-by0) x W pixels, and rank 0 stacks the stripes and crops the
top/bottom padding.  Results are identical to the single-GPU path on the
same frame (tests/test_stripes.py, tests/test_stripes_gpu.py).

The exchange is one gather of the coded stripes to rank 0 (shard.Group:
RCCL gatherv on GPU ranks, the host group in CPU tests).  Every rank is
handed the whole frame (or index array): it reads only its own rows.
"""
from __future__ import annotations

import numpy as np

from .. import dct as D
from .shard import frame_range


def block_rows(H: int, block_size: int, rank: int, world: int):
    """Block rows [by0, by1) of the padded frame coded by `rank`."""
    nby = (H + block_size - 1) // block_size
    return frame_range(nby, rank, world)


def _pad_top(H: int, block_size: int) -> int:
    Hp = (H + block_size - 1) // block_size * block_size
    return (Hp - H) // 2


def stripe_pixels(rgb: np.ndarray, by0: int, by1: int, block_size: int = 8) -> np.ndarray:
    """Rows [B*by0, B*by1) of the centred, zero-padded frame, at the frame's own width W."""
    H, W = rgb.shape[:2]
    B = block_size
    r0 = B * by0 - _pad_top(H, B)
    r1 = B * by1 - _pad_top(H, B)
    lo, hi = max(r0, 0), min(r1, H)
    if lo == r0 and hi == r1:
        return np.ascontiguousarray(rgb[lo:hi])
    out = np.zeros((r1 - r0, W, 3), np.uint8)
    if lo < hi:
        out[lo - r0:hi - r0] = rgb[lo:hi]
    return out


def _rows(nby: int, by0: int, by1: int, B: int, subbands: bool) -> np.ndarray:
    """Frame index rows holding the stripe's rows, in the stripe's own row order."""
    if not subbands:
        return np.arange(B * by0, B * by1)
    return (np.arange(B)[:, None] * nby + np.arange(by0, by1)[None, :]).reshape(-1)


def place_stripe(k: np.ndarray, ks: np.ndarray, by0: int, by1: int, block_size: int = 8,
                 flags: int = 0) -> None:
    """Write a coded stripe (B*nbs x Wp x 3) into the frame's index array (Hp x Wp x 3)."""
    nby = k.shape[0] // block_size
    k[_rows(nby, by0, by1, block_size, not flags & D.VCF_DCT_NO_SUBBANDS)] = ks


def take_stripe(k: np.ndarray, by0: int, by1: int, block_size: int = 8, flags: int = 0) -> np.ndarray:
    """The stripe's indices, laid out as a B*nbs x Wp x 3 frame of their own."""
    nby = k.shape[0] // block_size
    return np.ascontiguousarray(k[_rows(nby, by0, by1, block_size, not flags & D.VCF_DCT_NO_SUBBANDS)])


def encode_frame(rgb: np.ndarray, group, Q: int = 32, flags: int = 0, block_size: int = 8, encode=None):
    """Rank 0: the frame's Hp x Wp x 3 uint8 indices, equal to D.encode(rgb, ...); other ranks: None.

    `encode(stripe, Q, flags, block_size)` codes one stripe (default: the HIP kernels)."""
    rgb = np.asarray(rgb)
    if rgb.dtype != np.uint8 or rgb.ndim != 3 or rgb.shape[2] != 3:
        raise ValueError("Input image must be a 3D uint8 array (height, width, channels).")
    if not D.block_size_supported(block_size):
        raise NotImplementedError(f"-B {block_size} is not supported")
    H, W = rgb.shape[:2]
    B = block_size
    Hp, Wp = D.padded_shape(H, W, B)
    enc = encode or (lambda x, q, f, b: D.encode(x, q, f, block_size=b))
    by0, by1 = block_rows(H, B, group.rank, group.world)
    ks = enc(stripe_pixels(rgb, by0, by1, B), Q, flags, B) if by1 > by0 else np.zeros((0, Wp, 3), np.uint8)
    if ks.shape != (B * (by1 - by0), Wp, 3):
        raise RuntimeError(f"stripe coder returned {ks.shape}")
    blobs = group.gather_blobs(ks.tobytes())
    if group.rank != 0:
        return None
    k = np.empty((Hp, Wp, 3), np.uint8)
    for r, blob in enumerate(blobs):
        b0, b1 = block_rows(H, B, r, group.world)
        place_stripe(k, np.frombuffer(blob, np.uint8).reshape(B * (b1 - b0), Wp, 3), b0, b1, B, flags)
    return k


def decode_frame(k: np.ndarray, H: int, W: int, group, Q: int = 32, flags: int = 0, block_size: int = 8,
                 decode=None):
    """Rank 0: the H x W x 3 reconstruction, equal to D.decode(k, H, W, ...); other ranks: None.

    `decode(ks, h, W, Q, flags, block_size)` decodes one stripe (default: the HIP kernels)."""
    k = np.asarray(k)
    B = block_size
    if not D.block_size_supported(B):
        raise NotImplementedError(f"-B {B} is not supported")
    Hp, Wp = D.padded_shape(H, W, B)
    if k.dtype != np.uint8 or k.shape != (Hp, Wp, 3):
        raise ValueError(f"index array {k.dtype} {k.shape} does not match {(Hp, Wp, 3)} uint8 for {H}x{W}")
    dec = decode or (lambda x, h, w, q, f, b: D.decode(x, h, w, q, f, block_size=b))
    by0, by1 = block_rows(H, B, group.rank, group.world)
    h = B * (by1 - by0)
    px = dec(take_stripe(k, by0, by1, B, flags), h, W, Q, flags, B) if h else np.zeros((0, W, 3), np.uint8)
    if px.shape != (h, W, 3):
        raise RuntimeError(f"stripe decoder returned {px.shape}")
    blobs = group.gather_blobs(px.tobytes())
    if group.rank != 0:
        return None
    padded = np.concatenate([np.frombuffer(b, np.uint8).reshape(-1, W, 3) for b in blobs])
    top = _pad_top(H, B)
    return np.ascontiguousarray(padded[top:top + H])
