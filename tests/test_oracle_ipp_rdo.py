"""The IPP -R (RDO mode decision) restatement against the reference's own
class IPP (tests/golden/ipp_rdo.npz, made by make_golden_ipp_rdo.py under
the reference's python3.9/scipy 1.7.1; no GPU):

  * per block: the mode IPP.rdo_block_decision picks, both get_rate values and
    the distortion it returns, bit for bit, for 3 frame pairs x 4 lambdas;
  * whole GOPs: IPP.temporal_filter with rdo_lambda > 0 -- the mode maps, the
    mixed-mode frames handed to the spatial codec and the reconstructions --
    rebuilt from the oracle's pieces (block matching, compensation, RDO modes,
    the mixed frame and its reconstruction, the 2D-DCT round trip)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

MAN = json.load(open(os.path.join(GOLDEN, "manifest_ipp_rdo.json")))


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "ipp_rdo.npz"))


@pytest.mark.parametrize("case", MAN["block_cases"], ids=lambda c: c["name"])
def test_rdo_block_decisions_match_reference(gold, case):
    n = case["name"]
    cur, comp = gold[f"{n}_cur"], gold[f"{n}_comp"]
    for li, lam in enumerate(case["lambdas"]):
        modes, costs = O.ipp_rdo_modes(cur, comp, case["bs"], case["qss"], lam, with_costs=True)
        assert np.array_equal(modes, gold[f"{n}_l{li}_modes"]), lam
        rates = gold[f"{n}_l{li}_rates"]
        assert np.array_equal(costs[..., 1], rates[..., 0]) and np.array_equal(costs[..., 3], rates[..., 1])
        chosen_d = np.where(modes == 1, costs[..., 2], costs[..., 0])
        assert np.array_equal(chosen_d, gold[f"{n}_l{li}_dist"])


def rdo_loop(frames, gop, bs, sr, Q, lam):
    """IPP.temporal_filter (:397-575) with rdo_lambda > 0 from the oracle's pieces."""
    def rt(img):
        H, W = img.shape[:2]
        return O.decode_frame(O.encode_frame(img, Q), H, W, Q)
    recon, modes_all, coded = [], [], []
    for g0 in range(0, len(frames), gop):
        coded.append(frames[g0])
        ref = rt(frames[g0])
        recon.append(ref)
        for p in range(1, min(gop, len(frames) - g0)):
            cur = frames[g0 + p]
            mv = O.ipp_block_matching(ref, cur, bs, sr, False)
            comp = O.ipp_motion_compensate(ref, mv, bs)
            modes = O.ipp_rdo_modes(cur, comp, bs, Q, lam)
            res = O.ipp_rdo_residual(cur, comp, modes, bs)
            coded.append(res)
            ref = O.ipp_rdo_reconstruct(comp, rt(res), modes, bs)
            recon.append(ref)
            modes_all.append(modes)
    return recon, modes_all, coded


@pytest.mark.parametrize("case", MAN["seq_cases"], ids=lambda c: c["name"])
def test_rdo_gop_loop_matches_reference(gold, case):
    n = case["name"]
    frames = list(gold[f"{n}_frames"])
    recon, modes, coded = rdo_loop(frames, case["gop"], case["bs"], case["sr"], case["qss"], case["rdo_lambda"])
    assert np.array_equal(np.stack(modes), gold[f"{n}_modes"])
    assert np.array_equal(np.stack(coded), gold[f"{n}_coded"])
    assert np.array_equal(np.stack(recon), gold[f"{n}_recon"])
    assert sum(case["I_blocks"]) > 0   # the fixture exercises both modes
