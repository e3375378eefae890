"""The CPU oracle against the reference's own outputs (no GPU).

Pins oracle/vcf_oracle.c -- the checker every GPU test compares with -- to
the golden fixtures that tests/golden/make_golden.py captured by running the
reference's unmodified glue (src/2D-DCT.py encode_fn/decode_fn, YCoCg.py,
deadzone.py, TIFF.py) over scipy/pocketfft:

  * every committed case: indices bit-exact (encode) and reconstruction
    bit-exact (decode of the reference's indices);
  * the 512x512 cases (config C1), by SHA-256 of input, indices and output;
  * 8x8 pocketfft blocks: scipy.fftpack dct(dct(b.T).T) in fp32 and
    idct(idct(b.T).T) of int16 blocks (promoted to fp64), bit for bit.
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_params, golden_cases, load_case
from oracle import oracle as O


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _synth():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.synth


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_oracle_encode_decode_vs_reference(case):
    d = load_case(case)
    Q, flags = case_params(case)
    H, W = d["rgb"].shape[:2]
    k = O.encode_frame(d["rgb"], Q, flags)
    assert k.shape == tuple(case["k_shape"])
    assert np.array_equal(k, d["k"])
    assert np.array_equal(O.decode_frame(d["k"], H, W, Q, flags), d["decoded"])


def test_oracle_shape_bin_matches_reference():
    """{out_fn}_shape.bin = struct.pack('iii', H, W, C) (2D-DCT.py:285-286)."""
    import struct
    for case in golden_cases():
        d = load_case(case)
        assert bytes(d["shape_bin"]) == struct.pack("<iii", case["H"], case["W"], 3)


@pytest.mark.parametrize("name", ["smooth_512x512", "rand_512x512"])
def test_oracle_512_cases_by_hash(manifest, name):
    case = [c for c in manifest["big_cases"] if c["name"] == name][0]
    rgb = _synth()(case["kind"], case["H"], case["W"], case["seed"])
    assert _sha(rgb) == case["sha256"]["rgb"]
    k = O.encode_frame(rgb, 32, 0)
    assert _sha(k) == case["sha256"]["k"]
    assert _sha(O.decode_frame(k, case["H"], case["W"], 32, 0)) == case["sha256"]["decoded"]


def test_oracle_blocks_vs_pocketfft():
    b = np.load(os.path.join(GOLDEN, "blocks.npz"))
    # forward: axis 0 (columns) then axis 1 (rows), fp32
    x = b["fwd_in"]
    cols = O.dct2_8(np.swapaxes(x, 1, 2), np.float32)          # transform each column
    out = O.dct2_8(np.swapaxes(cols, 1, 2), np.float32)         # then each row
    assert np.array_equal(out.view(np.uint32), b["fwd_out"].view(np.uint32))
    # inverse: int16 blocks promote to float64
    y = b["inv_in"].astype(np.float64)
    cols = O.dct3_8(np.swapaxes(y, 1, 2), np.float64)
    out = O.dct3_8(np.swapaxes(cols, 1, 2), np.float64)
    assert np.array_equal(out.view(np.uint64), b["inv_out"].view(np.uint64))


def test_oracle_errors():
    with pytest.raises(ValueError):
        O.encode_frame(np.zeros((8, 8), np.uint8))
    with pytest.raises(ValueError):
        O.decode_frame(np.zeros((8, 16, 3), np.uint8), 8, 8)


def test_oracle_perceptual_weights_table():
    """-p tables of 2D-DCT.py:66-83 divided by 121 (luma) and 99 (chroma)."""
    w = O.perceptual_weights()
    assert w.shape == (3, 8, 8)
    assert w[0, 0, 0] == 16 / 121 and w[1, 7, 7] == 99 / 99 and w[2, 0, 1] == 18 / 99
