"""IPP -R (RDO mode decision) on the GPU (vcf_amd/csrc/vcf_ipp_rdo.hip through
the C ABI) against the reference's own class IPP (tests/golden/ipp_rdo.npz)
and the oracle; and the IPP CoDec with -R end to end: its mode maps, the
mixed-mode frames and the decoder's reconstructions equal the reference's
temporal_filter."""
import json
import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

MAN = json.load(open(os.path.join(GOLDEN, "manifest_ipp_rdo.json")))


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "ipp_rdo.npz"))


@pytest.fixture(scope="module")
def K():
    from vcf_amd import ipp
    return ipp


@pytest.mark.parametrize("case", MAN["block_cases"], ids=lambda c: c["name"])
def test_rdo_modes_match_reference(K, gold, case):
    n = case["name"]
    cur, comp = gold[f"{n}_cur"], gold[f"{n}_comp"]
    for li, lam in enumerate(case["lambdas"]):
        modes, costs = K.rdo_modes(cur, comp, case["bs"], case["qss"], lam, with_costs=True)
        assert np.array_equal(modes, gold[f"{n}_l{li}_modes"]), lam
        rates = gold[f"{n}_l{li}_rates"]
        assert np.array_equal(costs[..., 1], rates[..., 0]) and np.array_equal(costs[..., 3], rates[..., 1])
        chosen_d = np.where(modes == 1, costs[..., 2], costs[..., 0])
        assert np.array_equal(chosen_d, gold[f"{n}_l{li}_dist"])


def _pair(H, W, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    y, x = np.mgrid[0:H, 0:W]
    cur = np.stack([128 + 90 * np.sin(x / 9 + c) * np.cos(y / 5 - c) for c in range(3)], -1)
    cur = np.clip(np.rint(cur + rng.normal(0, 5, cur.shape)), 0, 255).astype(np.uint8)
    comp = cur.astype(np.int32) + rng.integers(-20, 21, cur.shape) * (rng.random((H, W, 1)) < 0.5)
    comp[: H // 2, : W // 3] = rng.integers(0, 256, comp[: H // 2, : W // 3].shape)
    return cur, np.clip(comp, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("bs", [2, 4, 8, 12, 16, 24, 32])
@pytest.mark.parametrize("Q,lam", [(32, 0.5), (7, 5.0), (64, 0.0)])
def test_rdo_modes_vs_oracle(K, bs, Q, lam):
    cur, comp = _pair(2 * bs + 5, 3 * bs + 2, bs * 13 + Q)
    m, c = K.rdo_modes(cur, comp, bs, Q, lam, with_costs=True)
    mo, co = O.ipp_rdo_modes(cur, comp, bs, Q, lam, with_costs=True)
    assert np.array_equal(m, mo)
    assert np.array_equal(c.view(np.uint64), co.view(np.uint64))
    res = K.rdo_residual(cur, comp, m, bs)
    assert np.array_equal(res, O.ipp_rdo_residual(cur, comp, m, bs))
    rec = _pair(cur.shape[0], cur.shape[1], 7)[0]
    assert np.array_equal(K.rdo_reconstruct(comp, rec, m, bs), O.ipp_rdo_reconstruct(comp, rec, m, bs))


def test_rdo_unsupported_block_size(K):
    cur, comp = _pair(40, 40, 1)
    with pytest.raises(NotImplementedError):
        K.rdo_modes(cur, comp, 5, 32, 1.0)


@pytest.mark.parametrize("case", MAN["seq_cases"], ids=lambda c: c["name"])
def test_ipp_codec_rdo_matches_reference(gold, case, tmp_path):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.ipp import CoDec
    n = case["name"]
    frames = gold[f"{n}_frames"]
    for i, f in enumerate(frames):
        Image.fromarray(f).save(str(tmp_path / f"in_{i:04d}.png"))
    pat = str(tmp_path / "in_%04d.png")
    enc, dec = str(tmp_path / "enc" / "v"), str(tmp_path / "dec" / "v")
    flags = ["-N", str(case["n"]), "-G", str(case["gop"]), "-M", str(case["bs"]), "-S", str(case["sr"]),
             "-q", str(case["qss"]), "-R", str(case["rdo_lambda"])]
    CoDec(P.parse(P.ipp_parser(), ["encode", "-i", pat, "-O", enc] + flags)).encode()
    with np.load(enc + "_mv.npz", allow_pickle=False) as z:
        assert np.array_equal(z["modes_u8"], gold[f"{n}_modes"])
        assert np.array_equal(z["mv_f32"], gold[f"{n}_mv"])
    d = CoDec(P.parse(P.ipp_parser(), ["decode", "-i", enc, "-O", dec, "-M", str(case["bs"]), "-q",
                                       str(case["qss"])]))
    assert d.decode() == case["n"]
    for i in range(case["n"]):
        got = np.asarray(Image.open(f"{dec}_{i:04d}.png").convert("RGB"))
        assert np.array_equal(got, gold[f"{n}_recon"][i]), f"frame {i}"
