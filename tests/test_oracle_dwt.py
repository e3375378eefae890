"""The 2D-DWT oracle (oracle/vcf_dwt_oracle.cpp) against the reference.

  * dwt_pywt.npz: pywt 1.1.1 wavedec2 / waverec2 (mode 'per') on random
    float64 planes, bit for bit (the convolution order of pywt's C code);
  * dwt_<case>.npz: the reference's src/2D-DWT.py encode_fn files (every
    subband's indices) and decode_fn output, bit for bit
    (tests/golden/make_golden_dwt.py)."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

_MAN = json.load(open(os.path.join(GOLDEN, "manifest_dwt.json")))
_SHORT = json.load(open(os.path.join(GOLDEN, "manifest_dwt_short.json")))


def _params(case):
    fl = case["flags"]
    w = fl[fl.index("-w") + 1] if "-w" in fl else "db5"
    Q = int(fl[fl.index("-q") + 1]) if "-q" in fl else 32
    return w, case["levels"], Q


def _pywt_tags():
    d = np.load(os.path.join(GOLDEN, "dwt_pywt.npz"))
    return sorted({m.group(1) for k in d.files for m in [re.match(r"fwd_in_(.*)", k)] if m})


@pytest.mark.parametrize("tag", _pywt_tags())
def test_wavedec2_waverec2_vs_pywt(tag):
    d = np.load(os.path.join(GOLDEN, "dwt_pywt.npz"))
    wname = tag.split("_")[0]
    L = int(tag.rsplit("_l", 1)[1])
    x = d[f"fwd_in_{tag}"]
    c = O.wavedec2(x, wname, L)
    assert np.array_equal(c[0], d[f"fwd_{tag}_0"])
    for l in range(1, L + 1):
        for s in range(3):
            assert np.array_equal(c[l][s], d[f"fwd_{tag}_{l}_{s}"]), (l, s)
    ci = [d[f"inv_{tag}_0"]] + [tuple(d[f"inv_{tag}_{l}_{s}"] for s in range(3)) for l in range(1, L + 1)]
    y = O.waverec2(ci, wname, *x.shape)
    ref = d[f"inv_out_{tag}"]
    assert y.shape == ref.shape and np.array_equal(y, ref)


@pytest.mark.parametrize("case", _MAN["cases"], ids=lambda c: c["name"])
def test_dwt_codec_vs_reference(case):
    d = np.load(os.path.join(GOLDEN, f"dwt_{case['name']}.npz"))
    w, L, Q = _params(case)
    sb = O.dwt_encode_frame(d["rgb"], w, L, Q)
    assert list(sb) == case["subbands"]
    for name in case["subbands"]:
        assert np.array_equal(sb[name], d[name]), name
    ref_sb = {n: d[n] for n in case["subbands"]}
    out = O.dwt_decode_frame(ref_sb, case["H"], case["W"], w, L, Q)
    assert list(out.shape) == case["decoded_shape"]
    assert np.array_equal(out, d["decoded"])


def test_wavelet_table():
    assert O.wavelet_index("db5") >= 0 and O.wavelet_index("bior4.4") >= 0
    with pytest.raises(ValueError):
        O.wavelet_index("nope")


def test_lines_shorter_than_the_filter_vs_pywt():
    """pywt's short-input branch: idwt/dwt of every line length 1 .. F/2 + 3 for all
    106 discrete wavelets, bit for bit (dwt_short_pywt.npz, make_golden_dwt_short.py)."""
    d = np.load(os.path.join(GOLDEN, "dwt_short_pywt.npz"))
    names = [str(n) for n in d["names"]]
    assert len(names) == 106
    n = 0
    for w in names:
        N = 1
        while f"inv_{w}_{N}" in d.files:
            y = O.idwt1(d[f"inv_a_{w}_{N}"], d[f"inv_d_{w}_{N}"], w)
            assert np.array_equal(y.view(np.uint64), d[f"inv_{w}_{N}"].view(np.uint64)), (w, N)
            cA, cD = O.dwt1(d[f"fwd_x_{w}_{N}"], w)
            assert np.array_equal(cA, d[f"fwd_a_{w}_{N}"]) and np.array_equal(cD, d[f"fwd_d_{w}_{N}"]), (w, N)
            N += 1
            n += 1
    assert n > 1000


@pytest.mark.parametrize("case", _SHORT["cases"], ids=lambda c: c["name"])
def test_dwt_codec_short_subbands_vs_reference(case):
    d = np.load(os.path.join(GOLDEN, case["file"]))
    w, L, Q = _params(case)
    sb = O.dwt_encode_frame(d["rgb"], w, L, Q)
    for name in case["subbands"]:
        assert np.array_equal(sb[name], d[name]), name
    out = O.dwt_decode_frame({n: d[n] for n in case["subbands"]}, case["H"], case["W"], w, L, Q)
    assert np.array_equal(out, d["decoded"])
