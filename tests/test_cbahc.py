"""CBAHC (src/CBAHC.py) on the host: the native coder writes the reference's
own .huf bit streams bit for bit (tests/golden/make_golden_cbahc.py ran the
unmodified reference) and decodes them."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from vcf_amd import cbahc as H

_MAN = json.load(open(os.path.join(GOLDEN, "manifest_cbahc.json")))


@pytest.mark.parametrize("case", _MAN["cases"], ids=lambda c: c["name"])
def test_stream_equals_reference(case):
    d = np.load(os.path.join(GOLDEN, "cbahc.npz"))
    sym = d[f"{case['name']}_sym"]
    data, nbits = H.encode_symbols(sym, case["order"])
    assert nbits == case["nbits"] == int(d[f"{case['name']}_nbits"][0])
    assert data == bytes(d[f"{case['name']}_huf"])
    assert np.array_equal(H.decode_symbols(data, nbits, sym.size, case["order"]), sym.ravel())


def test_codec_side_file(tmp_path):
    img = np.random.Generator(np.random.PCG64(4)).integers(100, 160, (9, 11, 3), dtype=np.uint8)
    c = H.CBAHCCodec(order=2)
    fn = str(tmp_path / "enc")
    b = c.compress(img, fn)
    assert os.path.exists(fn + "_adaptive_huffman_tree.pkl.gz")
    assert np.array_equal(c.decompress(b.getvalue(), fn), img)


@pytest.mark.parametrize("order", [0, 1, 3])
def test_round_trip_larger(order):
    rng = np.random.Generator(np.random.PCG64(order + 10))
    sym = np.clip(np.rint(rng.laplace(128, 2, 40000)), 0, 255).astype(np.uint8)
    data, nbits = H.encode_symbols(sym, order)
    assert np.array_equal(H.decode_symbols(data, nbits, sym.size, order), sym)


def test_truncated_stream_raises():
    data, nbits = H.encode_symbols(np.arange(200, dtype=np.uint8), 0)
    with pytest.raises(ValueError):
        H.decode_symbols(data, nbits - 5, 200, 0)
