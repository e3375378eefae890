"""A12: color_transforms.YCrCb = cv2.cvtColor(RGB2YCrCb / YCrCb2RGB) on uint8.

OpenCV's integer path (yuv_shift = 14, CV_DESCALE rounding, saturate_cast):
  Y  = (4899 R + 9617 G + 1868 B + 2^13) >> 14
  Cr = ((R - Y) 11682 + 128 * 2^14 + 2^13) >> 14
  Cb = ((B - Y)  9241 + 128 * 2^14 + 2^13) >> 14
  R = Y + ((Cr - 128) 22987 + 2^13) >> 14
  G = Y + ((Cb - 128) (-5636) + (Cr - 128) (-11698) + 2^13) >> 14
  B = Y + ((Cb - 128) 29049 + 2^13) >> 14,   each saturated to 0..255.
Unpinned: neither the package nor OpenCV is in this image.  With
VCF_GOLDEN_YCRCB_UNUSED=1 both functions raise, which make_golden_plugins.py
uses to show that 2D-DCT.py / 2D-DWT.py -t YCrCb never call them.
"""
import os

import numpy as np


def _guard():
    if os.environ.get("VCF_GOLDEN_YCRCB_UNUSED") == "1":
        raise AssertionError("color_transforms.YCrCb was called")


def from_RGB(img):
    _guard()
    a = np.asarray(img)
    assert a.dtype == np.uint8, a.dtype
    r, g, b = (a[..., i].astype(np.int64) for i in range(3))
    y = (r * 4899 + g * 9617 + b * 1868 + 8192) >> 14
    cr = ((r - y) * 11682 + (128 << 14) + 8192) >> 14
    cb = ((b - y) * 9241 + (128 << 14) + 8192) >> 14
    return np.clip(np.stack([y, cr, cb], -1), 0, 255).astype(np.uint8)


def to_RGB(img):
    _guard()
    a = np.asarray(img)
    assert a.dtype == np.uint8, a.dtype
    y, cr, cb = (a[..., i].astype(np.int64) for i in range(3))
    cr, cb = cr - 128, cb - 128
    r = y + ((cr * 22987 + 8192) >> 14)
    g = y + ((cb * -5636 + cr * -11698 + 8192) >> 14)
    b = y + ((cb * 29049 + 8192) >> 14)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)
