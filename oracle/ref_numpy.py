"""The reference's CPU path for the headline workload, restated in numpy/scipy.

TEST INFRASTRUCTURE ONLY (like everything under oracle/): imported by tests/
and by bench.py's cpu_baseline leg, never by the product path.

`encode_frame_loop` is reference-faithful: it runs src/2D-DCT.py encode_fn
(:276-361) with the stand-ins of SURVEY.md Appendix B for the un-vendored
packages, in the same order and dtypes:
- `astype(np.float32)` (:276), `pad_and_center_to_multiple_of_block_size`
  (:187-229, zero padding, extra row/column bottom/right);
- `img -= 128` (:292, offset of `-a deadzone`, :107-110);
- `from_RGB` (:298; A4: matrix YCoCg into `empty_like`, YCoCg.py:25-35);
- `space_analyze(CT_img, 8, 8)` (:303; A1: per block and channel
  `dct(dct(b.T, norm='ortho').T, norm='ortho')` with scipy.fftpack, a
  Python loop over the 3 x H/8 x W/8 blocks -- what makes the reference slow);
- `get_subbands` (:336; A3), `quantize_decom` (:343 -> deadzone.py:95-102;
  A5: `(x / Q).astype(np.int32)`), `decom_k += 128` (:348),
  `astype(np.uint8)` (:361, wraps modulo 256).

`encode_frame` computes the same indices with one scipy.fft call per axis
over the whole frame (bitwise equal to the per-block
idiom -- pocketfft runs the same length-8 transform either way) and
`workers` threads: the best this host's CPUs do on the reference's
arithmetic.

Both are pinned by tests/test_ref_numpy.py against the fixtures the
reference itself produced (tests/golden/dct_*.npz, manifest.json).
"""
from __future__ import annotations

import numpy as np

B = 8
OFFSET = 128


def _pad(img: np.ndarray, b: int = B) -> np.ndarray:
    """2D-DCT.py:187-229."""
    if img.ndim != 3:
        raise ValueError("Input image must be a 3D array (height, width, channels).")
    h, w = img.shape[:2]
    th, tw = (h + b - 1) // b * b, (w + b - 1) // b * b
    pt, pl = (th - h) // 2, (tw - w) // 2
    return np.pad(img, ((pt, th - h - pt), (pl, tw - w - pl), (0, 0)), mode="constant", constant_values=0)


def _from_rgb(rgb: np.ndarray) -> np.ndarray:
    """A4 (color_transforms.YCoCg.from_RGB, called at 2D-DCT.py:298)."""
    R, G, Bc = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    o = np.empty_like(rgb)
    o[..., 0] = R / 4 + G / 2 + Bc / 4
    o[..., 1] = R / 2 - Bc / 2
    o[..., 2] = -R / 4 + G / 2 - Bc / 4
    return o


def _get_subbands(img: np.ndarray, b: int = B) -> np.ndarray:
    """A3 (DCT2D.block_DCT.get_subbands, 2D-DCT.py:336)."""
    sy, sx = img.shape[0] // b, img.shape[1] // b
    out = np.empty_like(img)
    for i in range(b):
        for j in range(b):
            out[i * sy:(i + 1) * sy, j * sx:(j + 1) * sx] = img[i::b, j::b]
    return out


def _tail(dct_img: np.ndarray, Q: int, subbands: bool) -> np.ndarray:
    """2D-DCT.py:333-361 (no -p): subbands, deadzone, +128, uint8 wrap."""
    decom = _get_subbands(dct_img) if subbands else dct_img
    k = (decom / Q).astype(np.int32)          # deadzone.py:95-102 (A5)
    k += OFFSET                               # :348
    return k.astype(np.uint8)                 # :361


def encode_frame_loop(rgb: np.ndarray, Q: int = 32, subbands: bool = True) -> np.ndarray:
    """Reference-faithful encode_fn: per-block scipy.fftpack loop (A1), 1 core."""
    from scipy.fftpack import dct
    img = _pad(rgb.astype(np.float32))
    img -= OFFSET
    ct = _from_rgb(img)
    out = np.empty_like(ct)                   # output dtype = input dtype (A1)
    for y in range(0, ct.shape[0], B):
        for x in range(0, ct.shape[1], B):
            for c in range(ct.shape[2]):
                blk = ct[y:y + B, x:x + B, c]
                out[y:y + B, x:x + B, c] = dct(dct(blk.T, norm="ortho").T, norm="ortho")
    return _tail(out, Q, subbands)


def encode_frame(rgb: np.ndarray, Q: int = 32, subbands: bool = True, workers: int = 1) -> np.ndarray:
    """The same indices, the transform vectorised over the frame (scipy.fft, `workers` threads)."""
    import scipy.fft as sf
    img = _pad(rgb.astype(np.float32))
    img -= OFFSET
    ct = _from_rgb(img)
    H, W = ct.shape[:2]
    v = ct.reshape(H // B, B, W // B, B, 3)
    # dct(b.T).T transforms each block's columns (axis 1 of the view) first, then its rows (axis 3)
    v = sf.dct(v, axis=1, norm="ortho", workers=workers)
    v = sf.dct(v, axis=3, norm="ortho", workers=workers)
    return _tail(np.ascontiguousarray(v.reshape(H, W, 3)), Q, subbands)
