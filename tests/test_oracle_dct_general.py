"""The any-block-size CPU oracle against the reference's own outputs (no GPU).

Pins oracle/vcf_dct_general_oracle.cpp -- the checker the generic-B GPU tests
compare with -- to fixtures tests/golden/make_golden_general.py captured from
the reference:

  * scipy.fftpack (scipy 1.7.1, the reference's pocketfft) dct/idct with
    norm='ortho' for every covered length 1..128, bit for bit;
  * src/2D-DCT.py encode_fn/decode_fn (unmodified glue) at -B 1, 2, 3, 4,
    12, 16, 32, 64, 96, 128 (padding, -x, several -q): indices and
    reconstructions bit-exact;
  * lengths with a prime factor above 5 (pocketfft radfg/radbg) 1..200 vs
    scipy, and the reference's glue at -B 7, 11, 13, 14, 21, 49, 98, 130, 200
    (make_golden_radg.py); the Bluestein lengths pocketfft_r picks (fftblue
    over cfftp: scipy.fft c2c, scipy.fftpack dct/idct at all 67 lengths <= 600,
    the glue at -B 191 and 478, make_golden_blue.py);
  * the -L search (optimize_block_size, 2D-DCT.py:533-579): the codec's host
    logic (vcf_amd/codec/dct2d.py) with the oracle standing in for the GPU
    transforms reproduces the reference's J for every candidate block size
    and its choice.  The GPU run of the same search is in test_dct_any_gpu.py.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest_general.json")))


def _qf(flags):
    Q = int(flags[flags.index("-q") + 1]) if "-q" in flags else 32
    B = int(flags[flags.index("-B") + 1]) if "-B" in flags else 8
    return B, Q, (1 if "-x" in flags else 0)


@pytest.mark.parametrize("N", MANIFEST["lengths"])
def test_oracle_dct_lengths_vs_scipy(N):
    g = np.load(os.path.join(GOLDEN, "blocks_general.npz"))
    assert O.dct_supported(N)
    fwd = O.dct_n(g[f"fwd_in_{N}"], 2, np.float32)
    assert fwd.dtype == g[f"fwd_out_{N}"].dtype == np.float32
    assert np.array_equal(fwd.view(np.uint32), g[f"fwd_out_{N}"].view(np.uint32))
    inv = O.dct_n(g[f"inv_in_{N}"].astype(np.float64), 3, np.float64)
    assert np.array_equal(inv.view(np.uint64), g[f"inv_out_{N}"].view(np.uint64))


RADG = json.load(open(os.path.join(GOLDEN, "manifest_radg.json")))


@pytest.mark.parametrize("N", RADG["lengths"])
def test_oracle_dct_radfg_radbg_lengths_vs_scipy(N):
    """Lengths with a prime factor above 5 (pocketfft's generic radfg/radbg),
    against scipy.fftpack under the reference's python (make_golden_radg.py)."""
    g = np.load(os.path.join(GOLDEN, "blocks_radg.npz"))
    assert O.dct_supported(N)
    fwd = O.dct_n(g[f"fwd_in_{N}"], 2, np.float32)
    assert np.array_equal(fwd.view(np.uint32), g[f"fwd_out_{N}"].view(np.uint32))
    inv = O.dct_n(g[f"inv_in_{N}"].astype(np.float64), 3, np.float64)
    assert np.array_equal(inv.view(np.uint64), g[f"inv_out_{N}"].view(np.uint64))


def test_oracle_dct_bluestein_lengths():
    """pocketfft_r plans exactly these lengths 1..600 with Bluestein; the
    restatement covers them (fftblue over cfftp) and every rfftp length."""
    blue = set(RADG["bluestein_lengths"])
    assert blue and min(blue) == 191
    assert blue == set(BLUE["bluestein_lengths"])
    for N in range(1, 601):
        assert O.dct_supported(N), N
        assert O.dct_uses_bluestein(N) == (N in blue), N


BLUE = json.load(open(os.path.join(GOLDEN, "manifest_blue.json")))
PASSG = {13, 169}   # cfftp lengths with a prime factor above 11 (generic passg, not restated)


def test_oracle_cfft_vs_scipy():
    """cfftp (the complex FFT Bluestein runs on) against scipy.fft.fft/ifft
    under the reference's python (make_golden_blue.py), bit for bit: every
    padded length the Bluestein plans of N <= 600 use, plus small lengths that
    exercise each pass; ifft with norm='forward' is the unnormalised backward
    pass."""
    g = np.load(os.path.join(GOLDEN, "cfft_blue.npz"))
    for N in BLUE["cfft_lengths"]:
        for nm in ("c64", "c128"):
            x = g[f"x_{nm}_{N}"]
            if N in PASSG:
                with pytest.raises(ValueError):
                    O.cfft(x)
                continue
            assert np.array_equal(O.cfft(x, True), g[f"fwd_{nm}_{N}"]), (N, nm)
            assert np.array_equal(O.cfft(x, False), g[f"bwd_{nm}_{N}"]), (N, nm)


@pytest.mark.parametrize("N", BLUE["bluestein_lengths"])
def test_oracle_dct_bluestein_blocks_vs_scipy(N):
    """DCT-II/III of the Bluestein lengths (fftblue::exec_r inside T_dcst23)
    against scipy.fftpack under the reference's python, bit for bit."""
    g = np.load(os.path.join(GOLDEN, "blocks_blue.npz"))
    fwd = O.dct_n(g[f"fwd_in_{N}"], 2, np.float32)
    assert np.array_equal(fwd.view(np.uint32), g[f"fwd_out_{N}"].view(np.uint32))
    inv = O.dct_n(g[f"inv_in_{N}"].astype(np.float64), 3, np.float64)
    assert np.array_equal(inv.view(np.uint64), g[f"inv_out_{N}"].view(np.uint64))


@pytest.mark.parametrize("case", BLUE["cases"], ids=lambda c: c["name"])
def test_oracle_bluestein_block_sizes_vs_reference(case):
    """src/2D-DCT.py encode_fn/decode_fn at -B 191 and -B 478 (2 x 239)."""
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = O.encode_frame_b(d["rgb"], B, Q, flags)
    assert k.shape == tuple(case["k_shape"])
    assert np.array_equal(k, d["k"])
    assert np.array_equal(O.decode_frame_b(d["k"], H, W, B, Q, flags), d["decoded"])


@pytest.mark.parametrize("case", RADG["cases"], ids=lambda c: c["name"])
def test_oracle_radg_block_sizes_vs_reference(case):
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = O.encode_frame_b(d["rgb"], B, Q, flags)
    assert k.shape == tuple(case["k_shape"])
    assert np.array_equal(k, d["k"])
    assert np.array_equal(O.decode_frame_b(d["k"], H, W, B, Q, flags), d["decoded"])


@pytest.mark.parametrize("case", MANIFEST["cases"], ids=lambda c: c["name"])
def test_oracle_any_block_size_vs_reference(case):
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = O.encode_frame_b(d["rgb"], B, Q, flags)
    assert k.shape == tuple(case["k_shape"])
    assert np.array_equal(k, d["k"])
    assert np.array_equal(O.decode_frame_b(d["k"], H, W, B, Q, flags), d["decoded"])


def _args(lam, extra):
    from vcf_amd.codec import parser as P
    argv = ["encode", "-L", lam] + extra
    return P.dct_parser().parse_known_args(argv)[0]


@pytest.mark.parametrize("case", MANIFEST["L_cases"], ids=lambda c: c["name"])
def test_L_search_host_logic_with_oracle_transforms(case, monkeypatch):
    """optimize_block_size's rate/RMSE/J bookkeeping on the host, with the
    oracle's int32 analysis/synthesis in place of the GPU kernels."""
    import vcf_amd.codec.dct2d as C
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    rgb = d["rgb"]
    fl = case["flags"]
    Q = int(fl[fl.index("-q") + 1]) if "-q" in fl else 32
    monkeypatch.setattr(C.D, "encode_k32", lambda img, q, f, b: O.encode_frame_b(img, b, q, f, k32=True))
    monkeypatch.setattr(C.D, "decode_k32", lambda k, H, W, q, f, b: O.decode_frame_b(k, H, W, b, q, f))
    args = _args(fl[1], fl[2:])
    args.Lambda = None                       # construct without searching ...
    codec = C.CoDec(args)
    codec.Lambda = float(fl[1])
    assert codec.QSS == Q
    chosen = codec.optimize_block_size(rgb)  # ... then search this frame
    assert chosen == int(d["block_size"]) == case["chosen_block_size"]
    for b, j in zip(d["J_block_sizes"], d["J"]):
        assert codec.J[int(b)] == float(j), (b, codec.J[int(b)], float(j))
    # and the frame encode_fn then writes at the chosen size
    assert np.array_equal(O.encode_frame_b(rgb, chosen, Q, 0), d["k"])
