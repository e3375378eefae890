"""§8(f) row 4 plug-ins on the CPU: the oracle's restatement (oracle/plugins.py)
against the fixtures the reference's own glue produced (tests/golden/
plug_*.npz, make_golden_plugins.py), numpy 1.26's histogram arithmetic, the
library's host-side Lloyd-Max design against the oracle, and the parsers."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O
from oracle import plugins as P


def _manifest():
    with open(os.path.join(GOLDEN, "manifest_plugins.json")) as f:
        return json.load(f)


def _flag(fl, name, default):
    return int(fl[fl.index(name) + 1]) if name in fl else default


def cases(module=None):
    return [c for c in _manifest()["cases"] if module is None or c["module"] == module]


def load(case):
    return np.load(os.path.join(GOLDEN, f"plug_{case['name']}.npz"))


def params(case):
    fl = case["flags"]
    return dict(Q=_flag(fl, "-q", 32), lo=_flag(fl, "-m", 0), hi=_flag(fl, "-n", 255), B=_flag(fl, "-B", 8),
                flags=(1 if "-x" in fl else 0) | (2 if "-p" in fl else 0), lm="LloydMax" in fl)


def side_params(z):
    return bytes(z["params"]).decode()


@pytest.mark.parametrize("case", cases("2D-DCT"), ids=lambda c: c["name"])
def test_oracle_dct_lloydmax_matches_reference(case):
    z, p = load(case), params(case)
    rgb = z["rgb"]
    H, W = rgb.shape[:2]
    assert side_params(z) == f"{p['Q']}\n{p['lo']}\n{p['hi']}\n"
    coef = O.dct_raw_encode_b(rgb, p["B"], p["flags"])
    k, cents = P.lm_quantize(coef, p["Q"], p["lo"], p["hi"])
    assert k.dtype == np.float32                        # k = empty_like(decom) (LloydMax.py:96)
    assert np.array_equal(k.astype(np.uint8), z["k"])   # 2D-DCT.py:361
    for c in range(3):
        assert np.array_equal(cents[c], z[f"centroids_{c}"])
    y = P.lm_dequantize(z["k"].astype(np.int16), [z[f"centroids_{c}"] for c in range(3)])
    assert np.array_equal(O.dct_raw_decode_b(y, H, W, p["B"], p["flags"]), z["decoded"])


@pytest.mark.parametrize("case", cases("LloydMax"), ids=lambda c: c["name"])
def test_oracle_lloydmax_codec_matches_reference(case):
    z, p = load(case), params(case)
    k, cents = P.lm_quantize(z["rgb"], p["Q"], p["lo"], p["hi"])
    assert k.dtype == np.uint8 and np.array_equal(k, z["k"])
    for c in range(3):
        assert np.array_equal(cents[c], z[f"centroids_{c}"])
    assert np.array_equal(P.lm_dequantize(z["k"], cents), z["decoded"])


@pytest.mark.parametrize("case", cases("YCrCb"), ids=lambda c: c["name"])
def test_oracle_ycrcb_codec_matches_reference(case):
    z, p = load(case), params(case)
    assert z["k"].dtype == np.uint16
    if p["lm"]:
        x = P.ycrcb_from_rgb(z["rgb"]).astype(np.int16)
        k, cents = P.lm_quantize(x, p["Q"], p["lo"], p["hi"])
        assert np.array_equal(k.astype(np.uint16), z["k"])
        y = P.lm_dequantize(z["k"], cents).astype(np.int16).astype(np.uint8)
        assert np.array_equal(P.ycrcb_to_rgb(y), z["decoded"])
    else:
        assert np.array_equal(P.ycrcb_dz_encode(z["rgb"], p["Q"]), z["k"])
        assert np.array_equal(P.ycrcb_dz_decode(z["k"], p["Q"]), z["decoded"])


def test_t_ycrcb_is_ycocg_in_the_transform_codecs():
    """2D-DCT.py / 2D-DWT.py -t YCrCb wrote the same files as -t YCoCg, with the
    YCrCb functions raising if called (make_golden_plugins.py same_case)."""
    same = _manifest()["same_as_ycocg"]
    assert {s["module"] for s in same} == {"2D-DCT", "2D-DWT"}
    assert all(s["equal"] for s in same)


RANGES = [(0, 255), (-2048, 2047), (-512, 511), (16, 200), (-3, 3)]


@pytest.mark.parametrize("i", range(len(RANGES)))
def test_oracle_histogram_is_numpy_126(i):
    z = np.load(os.path.join(GOLDEN, "plug_histograms.npz"))
    lo, hi = RANGES[i]
    for t in ("f32", "i16", "u8"):
        if f"{t}_x_{i}" in z.files:
            assert np.array_equal(P.histogram(z[f"{t}_x_{i}"], lo, hi), z[f"{t}_h_{i}"]), t


def test_library_design_equals_oracle():
    """vcf_lm_design is host code in libvcf_amd.so (no GPU needed)."""
    from vcf_amd import plugins as V
    rng = np.random.Generator(np.random.PCG64(5))
    for _ in range(200):
        lo = int(rng.integers(-3000, 300))
        L = int(rng.integers(1, 5000))
        Q = int(rng.integers(1, 300))
        counts = rng.integers(0, 1000, L) * (rng.random(L) < rng.random()) + 1
        assert np.array_equal(V.lm_design(counts, Q, lo), P.lloydmax_design(counts, Q, lo))
        assert V.lm_levels(Q, lo, lo + L - 1) == P.levels(Q, lo, lo + L - 1)
    for case in cases():
        z, p = load(case), params(case)
        if "centroids_0" in z.files:
            assert len(z["centroids_0"]) == V.lm_levels(p["Q"], p["lo"], p["hi"])


def test_library_design_rejects_bad_input():
    from vcf_amd import _lib, plugins as V
    with pytest.raises(_lib.VCFInvalidArgument):
        V.lm_design(np.zeros(10, np.int64), 2, 0)          # the glue's +1 guarantees no empty bin
    with pytest.raises(_lib.VCFInvalidArgument):
        V.lm_levels(0, 0, 255)
    with pytest.raises(_lib.VCFInvalidArgument):
        V.lm_levels(4, 10, 9)
    with pytest.raises(_lib.VCFUnsupported):
        V.lm_levels(4, 0, 70000)


def test_parsers_follow_the_quantizer_module():
    from vcf_amd.codec import parser as PP
    a = PP.parse(PP.dct_parser(quantizer=PP.quantizer_of(["encode", "-a", "LloydMax"])),
                 ["encode", "-a", "LloydMax", "-m", "-2048", "-n", "2047", "-q", "16"])
    assert (a.quantizer, a.min_val, a.max_val, a.QSS) == ("LloydMax", -2048, 2047, 16)
    d = PP.parse(PP.dct_parser(), ["encode"])
    assert not hasattr(d, "min_val")                     # deadzone.py adds no -m/-n
    a = PP.parse(PP.lloydmax_parser(), ["decode", "-q", "64", "-f", "no_filter"])
    assert (a.QSS, a.min_val, a.max_val, a.filter) == (64, 0, 255, "no_filter")
    a = PP.parse(PP.ycrcb_parser(), ["encode", "-q", "5"])
    assert (a.quantizer, a.QSS, a.entropy_image_codec) == ("deadzone", 5, "TIFF")


def test_codecs_accept_the_plugins_and_refuse_the_rest():
    from vcf_amd.codec import parser as PP
    from vcf_amd.codec.dct2d import CoDec
    from vcf_amd.codec.dwt2d import CoDec as DWTCoDec
    CoDec(PP.parse(PP.dct_parser(), ["encode", "-t", "YCrCb"]))
    DWTCoDec(PP.parse(PP.dwt_parser(), ["encode", "-t", "YCrCb"]))
    c = CoDec(PP.parse(PP.dct_parser(quantizer="LloydMax"), ["encode", "-a", "LloydMax"]))
    assert c.offset == 0 and c.lm is not None
    with pytest.raises(NotImplementedError):
        CoDec(PP.parse(PP.dct_parser(), ["encode", "-t", "color-DCT"]))
    with pytest.raises(NotImplementedError):
        CoDec(PP.parse(PP.dct_parser(), ["encode", "-a", "VQ"]))
    with pytest.raises(NotImplementedError):
        CoDec(PP.parse(PP.dct_parser(quantizer="LloydMax"), ["encode", "-a", "LloydMax", "-L", "1"]))
    with pytest.raises(NotImplementedError):
        c.encode_indices(np.zeros((8, 8, 3), np.uint8))


def test_dwt_codec_lifting_opt_in(monkeypatch):
    """The opt-in lifting form (no reference counterpart): VCF_DWT_LIFTING=1 or
    args.dwt_lifting; bior4.4 only, refused for any other wavelet."""
    from vcf_amd.codec import parser as PP
    from vcf_amd.codec.dwt2d import CoDec as DWTCoDec
    assert not DWTCoDec(PP.parse(PP.dwt_parser(), ["encode", "-w", "bior4.4"])).lifting
    monkeypatch.setenv("VCF_DWT_LIFTING", "1")
    assert DWTCoDec(PP.parse(PP.dwt_parser(), ["encode", "-w", "bior4.4"])).lifting
    with pytest.raises(NotImplementedError):
        DWTCoDec(PP.parse(PP.dwt_parser(), ["encode"]))   # the reference's default -w db5
    monkeypatch.delenv("VCF_DWT_LIFTING")
    args = PP.parse(PP.dwt_parser(), ["encode", "-w", "bior4.4"])
    args.dwt_lifting = True
    assert DWTCoDec(args).lifting
