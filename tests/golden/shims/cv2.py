"""A9: the few OpenCV calls the hot path makes, over PIL (lossless 8-bit RGB)."""
import numpy as np
from PIL import Image

IMREAD_UNCHANGED = -1
COLOR_BGR2RGB = 4
COLOR_RGB2BGR = 4
COLOR_RGB2GRAY = 7
INTER_AREA = 3
INTER_LINEAR = 1


def imread(fn, flag=-1):
    return np.array(Image.open(fn))[..., ::-1].copy()


def cvtColor(img, code):
    if code == COLOR_RGB2GRAY:   # OpenCV fixed-point: (R*4899 + G*9617 + B*1868 + 8192) >> 14
        i = img.astype(np.int32)
        return ((i[..., 0] * 4899 + i[..., 1] * 9617 + i[..., 2] * 1868 + 8192) >> 14).astype(np.uint8)
    return img[..., ::-1].copy()


def resize(img, size, interpolation=INTER_LINEAR):
    if tuple(size) == (img.shape[1], img.shape[0]):
        return img.copy()        # same-size resize is the identity in OpenCV
    raise NotImplementedError("shim resize only supports B=8 (identity)")
