"""A1-A3: DCT2D.block_DCT as the in-tree idiom of src/IPP_DCT.py:257-263."""
import numpy as np
from scipy.fftpack import dct, idct


def _fwd(b):
    return dct(dct(b.T, norm='ortho').T, norm='ortho')


def _inv(b):
    return idct(idct(b.T, norm='ortho').T, norm='ortho')


def _blockwise(img, by, bx, f):
    out = np.empty_like(img)          # output dtype = input dtype (A2)
    for y in range(0, img.shape[0], by):
        for x in range(0, img.shape[1], bx):
            for c in range(img.shape[2]):
                out[y:y + by, x:x + bx, c] = f(img[y:y + by, x:x + bx, c])
    return out


def analyze_image(img, by, bx):
    return _blockwise(img, by, bx, _fwd)


def synthesize_image(img, by, bx):
    return _blockwise(img, by, bx, _inv)


def get_subbands(img, by, bx):
    sy, sx = img.shape[0] // by, img.shape[1] // bx
    out = np.empty_like(img)
    for i in range(by):
        for j in range(bx):
            out[i * sy:(i + 1) * sy, j * sx:(j + 1) * sx] = img[i::by, j::bx]
    return out


def get_blocks(img, by, bx):
    sy, sx = img.shape[0] // by, img.shape[1] // bx
    print(sy, sx)                     # the notebook output "36 44" (III.ipynb cell 13)
    out = np.empty_like(img)
    for i in range(by):
        for j in range(bx):
            out[i::by, j::bx] = img[i * sy:(i + 1) * sy, j * sx:(j + 1) * sx]
    return out
