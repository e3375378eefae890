"""A4: matrix YCoCg into empty_like(input)."""
import numpy as np


def from_RGB(RGB):
    R, G, B = RGB[..., 0], RGB[..., 1], RGB[..., 2]
    o = np.empty_like(RGB)
    o[..., 0] = R / 4 + G / 2 + B / 4
    o[..., 1] = R / 2 - B / 2
    o[..., 2] = -R / 4 + G / 2 - B / 4
    return o


def to_RGB(YCoCg):
    Y, Co, Cg = YCoCg[..., 0], YCoCg[..., 1], YCoCg[..., 2]
    o = np.empty_like(YCoCg)
    o[..., 0] = Y + Co - Cg
    o[..., 1] = Y + Cg
    o[..., 2] = Y - Co - Cg
    return o
