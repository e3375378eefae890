"""The reference's stand-alone codecs (src/YCoCg.py, deadzone.py, TIFF.py,
CBAAC.py --order, CBAHC.py --order) without a GPU: the oracle's restatements
(oracle/plugins.py) against the fixtures the reference itself wrote
(tests/golden/sa_*.npz, make_golden_standalone.py), the host entropy codecs
(native CBAAC/CBAHC coders, the TIFF writer) reproducing the reference's
files byte for byte, and the CLI surface (parsers, --order).  The GPU
kernels are tests/test_standalone_gpu.py."""
import argparse
import json
import os

import numpy as np
import pytest
from PIL import Image

from oracle import plugins as O
from vcf_amd.codec import parser as P

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def cases(module=None):
    m = json.load(open(os.path.join(GOLD, "manifest_standalone.json")))
    return [c for c in m["cases"] if module is None or c["module"] in module]


def load(c):
    return np.load(os.path.join(GOLD, f"sa_{c['name']}.npz"), allow_pickle=False)


def qss(c):
    fl = c["flags"]
    return int(fl[fl.index("-q") + 1]) if "-q" in fl else 32


def order(c):
    fl = c["flags"]
    return int(fl[fl.index("--order") + 1]) if "--order" in fl else 0


@pytest.mark.parametrize("c", cases(("YCoCg", "deadzone")), ids=lambda c: c["name"])
def test_oracle_equals_reference(c):
    z = load(c)
    Q = qss(c)
    if c["module"] == "deadzone":
        assert np.array_equal(O.dz_u8_encode(z["rgb"], Q), z["k"])
        assert np.array_equal(O.dz_u8_decode(z["k"], Q), z["decoded"])
    elif "LloydMax" in c["flags"]:
        k, cents = O.ycocg_lm_encode(z["rgb"], Q, 0, 255)
        assert np.array_equal(k, z["k"])
        assert np.array_equal(O.ycocg_lm_decode(z["k"], cents), z["decoded"])
    else:
        assert np.array_equal(O.ycocg_dz_encode(z["rgb"], Q), z["k"])
        assert np.array_equal(O.ycocg_dz_decode(z["k"], Q), z["decoded"])


def test_oracle_ycocg_wraps_like_numpy():
    """Every u8 RGB triple (subsampled) through the oracle's integer form vs numpy's float64 glue."""
    g = np.arange(0, 256, 5, dtype=np.uint8)
    rgb = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 1, 3)
    a = rgb.astype(np.int16)
    R, G, B = (a[..., i].astype(np.int64) for i in range(3))
    y = np.stack([(R + 2 * G + B) // 4, np.trunc((R - B) / 2), np.trunc((-R + 2 * G - B) / 4)], -1)
    assert np.array_equal(O.ycocg_i16(rgb), y.astype(np.int16))
    for Q in (1, 3, 32, 255, 1000, 32767):
        k = O.ycocg_dz_encode(rgb, Q)
        assert np.array_equal(O.ycocg_dz_decode(k, Q).shape, rgb.shape)


def _codec(module, sub, flags):
    from vcf_amd.codec import pixel as X
    if module == "TIFF":
        return X.TIFFImageCoDec(P.parse(P.tiff_parser(), [sub] + flags))
    if module == "CBAAC":
        return X.CBAACImageCoDec(P.parse(P.cbaac_parser(), [sub] + flags))
    return X.CBAHCImageCoDec(P.parse(P.cbahc_parser(), [sub] + flags))


@pytest.mark.parametrize("c", cases(("TIFF", "CBAAC", "CBAHC")), ids=lambda c: c["name"])
def test_entropy_codecs_reproduce_reference_files(tmp_path, c):
    """encode_fn/decode_fn of the stand-alone entropy codecs: the encoded
    file equals the reference's byte for byte (CBAAC under assumption A8),
    CBAHC's side file holds the reference's shape/order/nbits, decoding the
    reference's file gives its decoded image."""
    z = load(c)
    src = str(tmp_path / "original.png")
    Image.fromarray(z["rgb"]).save(src)
    enc = _codec(c["module"], "encode", c["flags"])
    out = str(tmp_path / "encoded")
    if c["module"] == "CBAHC":
        enc.compress = lambda img, fn=out: enc.entropy.compress(img, out)   # side file beside the output
    n = enc.encode_fn(src, out)
    got = open(out + enc.file_extension, "rb").read()
    assert got == z["enc"].tobytes() and n == z["enc"].size
    dec = _codec(c["module"], "decode", c["flags"])
    if c["module"] == "CBAHC":
        import gzip
        with gzip.open(f"{out}_adaptive_huffman_tree.pkl.gz", "rb") as f:
            assert tuple(np.load(f, allow_pickle=False)) == tuple(z["side_shape"])
        dec.decompress = lambda cs, fn=out: dec.entropy.decompress(cs, out)
    dst = str(tmp_path / "decoded.png")
    dec.decode_fn(out, dst)
    assert np.array_equal(np.array(Image.open(dst)), z["decoded"])


def test_compress_fn_names():
    """CBAAC.py:81/97 and CBAHC.py:169/226 expose compress_fn/decompress_fn(img|bytes, fn)."""
    from vcf_amd.cbaac import CBAACCodec
    from vcf_amd.cbahc import CBAHCCodec
    z = load(cases(("CBAAC",))[1])
    c = CBAACCodec(1)
    b = c.compress_fn(z["rgb"], "/tmp/unused")
    assert b.getvalue() == z["enc"].tobytes()
    assert np.array_equal(c.decompress_fn(b.getvalue(), "/tmp/unused"), z["rgb"])
    assert callable(CBAHCCodec.compress_fn) and callable(CBAHCCodec.decompress_fn)


def test_parsers_and_order():
    ns = P.parse(P.cbaac_parser(), ["encode", "--order", "1"])
    assert ns.order == 1 and ns.original == "/tmp/original.png" and ns.encoded == "/tmp/encoded"
    ns = P.parse(P.cbahc_parser(), ["decode", "--order", "2"])
    assert ns.order == 2 and ns.decoded == "/tmp/decoded.png"
    ns = P.parse(P.ycocg_parser(), ["encode", "-q", "7"])
    assert (ns.quantizer, ns.QSS, ns.entropy_image_codec) == ("deadzone", 7, "TIFF")
    ns = P.parse(P.ycocg_parser(quantizer="LloydMax"), ["encode", "-a", "LloydMax", "-m", "-3"])
    assert ns.min_val == -3 and ns.max_val == 255
    ns = P.parse(P.deadzone_parser(), ["decode", "-f", "no_filter"])
    assert ns.filter == "no_filter" and ns.QSS == 32
    assert not hasattr(P.parse(P.tiff_parser(), ["encode"]), "QSS")
    # -c CBAHC brings CBAHC.py's --order into every codec chain (CBAHC.py:13-16 at import);
    # -c CBAAC does not (CBAAC.py adds it only as a program, :158-164)
    argv = ["encode", "-c", "CBAHC", "--order", "1"]
    assert P.parse(P.dct_parser(entropy=P.entropy_of(argv)), argv).order == 1
    argv = ["encode", "-c", "CBAAC", "--order", "1"]
    assert not hasattr(P.parse(P.dct_parser(entropy=P.entropy_of(argv)), argv), "order")
    assert P.entropy_of(["-g", "encode"]) == "TIFF"


def test_cbahc_order_reaches_the_dct_codec():
    from vcf_amd.codec.dct2d import make_entropy
    ns = argparse.Namespace(entropy_image_codec="CBAHC", order=1)
    assert make_entropy(ns).order == 1
