"""Test infrastructure (checker only): the opt-in lifting DWT's float64
coefficients against pywt's, restated by the oracle (oracle/vcf_dwt_oracle.cpp,
pywt 1.1.1 'per' wavedec2 of the int16 YCoCg planes, 2D-DWT.py:59-64).
Measured in the north star's unit (ULP of float64) and as absolute error."""
import numpy as np

from oracle import oracle as O


def ycocg_planes(rgb: np.ndarray):
    """A4's int16 YCoCg as 2D-DWT.py:59-62 feeds DWT2D: (R + 2G + B) >> 2,
    (R - B) / 2 and (2G - R - B) / 4 truncated toward zero, as float64."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    y = (r + 2 * g + b) >> 2
    co = np.fix((r - b) / 2)
    cg = np.fix((2 * g - r - b) / 4)
    return [np.asarray(p, np.float64) for p in (y, co, cg)]


def _ordered(x: np.ndarray) -> np.ndarray:
    """float64 -> int64 whose differences count ULPs (sign-magnitude to two's complement)."""
    i = x.view(np.int64)
    return np.where(i < 0, np.int64(-0x8000000000000000) - i, i)


def compare(got, rgb: np.ndarray, levels: int) -> dict:
    """got: vcf_amd.dwt.lift_coefficients(rgb, levels).  Per subband kind: max
    ULP distance over coefficients with |ref| >= 1 (near zero an ULP is
    meaningless), max absolute error, and that error relative to the
    subband's largest magnitude."""
    out = {"ulp_max": 0, "ulp_p99": 0.0, "abs_max": 0.0, "rel_to_subband_max": 0.0, "coefficients": 0,
           "bitwise_equal_frac": 0.0}
    eq = tot = 0
    ulps = []
    for c, plane in enumerate(ycocg_planes(rgb)):
        ref = O.wavedec2(plane, "bior4.4", levels)
        pairs = [(ref[0], got[c][0])] + [(a, b) for lv in range(1, levels + 1) for a, b in zip(ref[lv], got[c][lv])]
        for a, b in pairs:
            a = np.ascontiguousarray(a)
            b = np.ascontiguousarray(b)
            d = np.abs(a - b)
            out["abs_max"] = max(out["abs_max"], float(d.max()))
            scale = float(np.abs(a).max()) or 1.0
            out["rel_to_subband_max"] = max(out["rel_to_subband_max"], float(d.max()) / scale)
            big = np.abs(a) >= 1.0
            if big.any():
                u = np.abs(_ordered(a[big]) - _ordered(b[big]))
                out["ulp_max"] = max(out["ulp_max"], int(u.max()))
                ulps.append(u)
            eq += int(np.count_nonzero(a == b))
            tot += a.size
    out["coefficients"] = tot
    out["bitwise_equal_frac"] = round(eq / tot, 6)
    if ulps:
        out["ulp_p99"] = float(np.percentile(np.concatenate(ulps), 99))
    return out
