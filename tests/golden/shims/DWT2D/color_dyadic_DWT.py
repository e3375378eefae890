"""A6: per-channel pywt.wavedec2/waverec2, mode 'per', repacked per subband."""
import numpy as np
import pywt


def analyze(img, wavelet, levels):
    d = [pywt.wavedec2(img[..., c], wavelet=wavelet, level=levels, mode='per')
         for c in range(img.shape[2])]
    out = [np.stack([d[c][0] for c in range(img.shape[2])], -1)]
    for l in range(1, levels + 1):
        out.append(tuple(np.stack([d[c][l][s] for c in range(img.shape[2])], -1)
                         for s in range(3)))
    return out


def synthesize(decom, wavelet, levels):
    chans = []
    for c in range(decom[0].shape[-1]):
        co = [decom[0][..., c]] + [tuple(sb[..., c] for sb in r) for r in decom[1:]]
        chans.append(pywt.waverec2(co, wavelet=wavelet, mode='per'))
    return np.stack(chans, -1)
