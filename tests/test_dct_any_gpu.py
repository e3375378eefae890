"""GPU parity of the generic-block-size DCT+deadzone kernels (vcf_dct_any.hip)
and of the -L search, through the C ABI.

Bit-exact against (1) the reference's own encode_fn/decode_fn outputs at
-B 1..128 and its optimize_block_size choices and J values
(tests/golden/make_golden_general.py) and (2) the any-B oracle
(oracle/vcf_dct_general_oracle.cpp) on seeded sweeps: every covered block
size, padding, -x, Q in {1, 5, 32}, both index types (encode_fn's wrapped
uint8 / int16 and the -L search's int32), multi-frame batches.
"""
import json
import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

D = pytest.importorskip("vcf_amd.dct")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest_general.json")))
RADG = json.load(open(os.path.join(GOLDEN, "manifest_radg.json")))
LENGTHS = [1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 15, 16, 18, 20, 24, 25, 27, 30, 32, 36, 40, 45, 48, 50, 54, 60, 64, 72, 75, 80, 81, 90, 96, 100, 108, 120, 125, 128]


def _qf(flags):
    Q = int(flags[flags.index("-q") + 1]) if "-q" in flags else 32
    B = int(flags[flags.index("-B") + 1]) if "-B" in flags else 8
    return B, Q, (1 if "-x" in flags else 0)


def _smooth(H, W, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    y, x = np.mgrid[0:H, 0:W]
    v = np.stack([128 + 100 * np.sin(x / 13 + c) * np.cos(y / 7 - c) for c in range(3)], -1)
    return np.clip(np.rint(v + rng.normal(0, 6, (H, W, 3))), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("case", MANIFEST["cases"], ids=lambda c: c["name"])
def test_any_block_size_matches_reference_golden(case):
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = D.encode(d["rgb"], Q, flags, block_size=B)
    assert np.array_equal(k, d["k"])
    assert np.array_equal(D.decode(d["k"], H, W, Q, flags, block_size=B), d["decoded"])


@pytest.mark.parametrize("B", LENGTHS)
@pytest.mark.parametrize("Q,flags", [(32, 0), (5, 1), (1, 0)])
def test_any_block_size_vs_oracle(B, Q, flags):
    H, W = 2 * B + 5 if B < 64 else B + 3, 3 * B - 1 if B > 1 else 9
    rgb = _smooth(H, W, B * 31 + Q) if Q != 5 else np.random.default_rng(B).integers(0, 256, (H, W, 3), np.uint8)
    k = D.encode(rgb, Q, flags, block_size=B)
    assert np.array_equal(k, O.encode_frame_b(rgb, B, Q, flags))
    assert np.array_equal(D.decode(k, H, W, Q, flags, block_size=B), O.decode_frame_b(k, H, W, B, Q, flags))


@pytest.mark.parametrize("B", [2, 16, 128])
def test_any_block_size_batched_frames(B):
    frames = np.stack([_smooth(130, 260, s) for s in range(3)])
    k = D.encode(frames, 32, 0, block_size=B)
    for i in range(3):
        assert np.array_equal(k[i], O.encode_frame_b(frames[i], B, 32, 0))
    out = D.decode(k, 130, 260, 32, 0, block_size=B)
    for i in range(3):
        assert np.array_equal(out[i], O.decode_frame_b(k[i], 130, 260, B, 32, 0))


@pytest.mark.parametrize("B", [2, 4, 8, 32, 128])
@pytest.mark.parametrize("Q", [32, 3])
def test_k32_analysis_synthesis_vs_oracle(B, Q):
    """The -L search's own int32 path (no uint8 wrap, offset 0)."""
    rgb = _smooth(128 + (B == 4) * 8, 256, B + Q)
    H, W = rgb.shape[:2]
    k = D.encode_k32(rgb, Q, 0, block_size=B)
    assert k.dtype == np.int32
    assert np.array_equal(k, O.encode_frame_b(rgb, B, Q, 0, k32=True))
    if B == 128 and Q == 3:
        assert np.abs(k).max() > 127   # the wrap the uint8 path would apply is absent here
    assert np.array_equal(D.decode_k32(k, H, W, Q, 0, block_size=B), O.decode_frame_b(k, H, W, B, Q, 0))


def test_generic_kernels_equal_fused_8x8():
    rgb = _smooth(72, 136, 5)
    for flags in (0, 1):
        k8 = D.encode(rgb, 32, flags)
        assert np.array_equal(D.encode(rgb, 32, flags, variant=-1), k8)
        assert np.array_equal(D.decode(k8, 72, 136, 32, flags, variant=-1), D.decode(k8, 72, 136, 32, flags))


@pytest.mark.parametrize("case", MANIFEST["L_cases"], ids=lambda c: c["name"])
def test_L_search_matches_reference(case, tmp_path, monkeypatch):
    """CoDec(-L lambda) on the GPU picks the reference's block size with the
    reference's J for every candidate, then encode_fn writes its .tif."""
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    src = str(tmp_path / "original.png")
    Image.fromarray(d["rgb"]).save(src)
    monkeypatch.setattr(CoDec, "encode_read", lambda self, fn=src: self.encode_read_fn(fn))
    codec = CoDec(P.parse(P.dct_parser(), ["encode"] + case["flags"]))
    assert codec.block_size == case["chosen_block_size"]
    for b, j in zip(d["J_block_sizes"], d["J"]):
        assert codec.J[int(b)] == float(j)
    out = str(tmp_path / "encoded")
    codec.encode_fn(src, out)
    assert open(out + ".tif", "rb").read() == bytes(d["tif"])


@pytest.mark.parametrize("case", [c for c in MANIFEST["cases"] if c["name"].startswith(("b16", "b4_"))],
                         ids=lambda c: c["name"])
def test_codec_block_size_files_match_reference(case, tmp_path):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    src = str(tmp_path / "in.png")
    Image.fromarray(d["rgb"]).save(src)
    out = str(tmp_path / "encoded")
    n = CoDec(P.parse(P.dct_parser(), ["encode"] + case["flags"])).encode_fn(src, out)
    assert open(out + ".tif", "rb").read() == bytes(d["tif"]) and n == case["encode_bytes"]
    dec = str(tmp_path / "dec.png")
    CoDec(P.parse(P.dct_parser(), ["decode"] + case["flags"])).decode_fn(out, dec)
    assert np.array_equal(np.asarray(Image.open(dec).convert("RGB")), d["decoded"])


def test_unsupported_block_sizes_raise():
    from vcf_amd._lib import VCFUnsupported
    rgb = _smooth(20, 20, 0)
    for B in (4097, 5000):   # beyond the run-time path's 4096
        assert not D.block_size_supported(B)
        with pytest.raises(VCFUnsupported):
            D.encode(rgb, 32, 0, block_size=B)


# ---- the run-time-length path (vcf_pocketfft_rt.h): prime factors above 5, B > 128 ----

@pytest.mark.parametrize("case", RADG["cases"], ids=lambda c: c["name"])
def test_radg_block_size_matches_reference_golden(case):
    """The reference's own encode_fn/decode_fn at -B 7, 11, 13, 14, 21, 49, 98,
    130, 200 (tests/golden/make_golden_radg.py), bit for bit."""
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = D.encode(d["rgb"], Q, flags, block_size=B)
    assert np.array_equal(k, d["k"])
    assert np.array_equal(D.decode(d["k"], H, W, Q, flags, block_size=B), d["decoded"])


RT_LENGTHS = [7, 11, 13, 14, 17, 22, 33, 49, 63, 97, 127, 131, 154, 180, 256, 300, 343]


@pytest.mark.parametrize("B", RT_LENGTHS)
@pytest.mark.parametrize("Q,flags", [(32, 0), (5, 1)])
def test_runtime_block_size_vs_oracle(B, Q, flags):
    H, W = B + 3, 2 * B - 1
    rng = np.random.default_rng(B * 7 + Q)
    rgb = _smooth(H, W, B) if Q == 32 else rng.integers(0, 256, (H, W, 3), np.uint8)
    k = D.encode(rgb, Q, flags, block_size=B)
    assert np.array_equal(k, O.encode_frame_b(rgb, B, Q, flags))
    assert np.array_equal(D.decode(k, H, W, Q, flags, block_size=B), O.decode_frame_b(k, H, W, B, Q, flags))


@pytest.mark.parametrize("B", [7, 49, 130])
def test_runtime_block_size_int32_and_batches(B):
    """The int32 (-L style) index type and multi-frame launches on the run-time path."""
    H, W = 2 * B + 1, B + 4
    frames = np.stack([_smooth(H, W, s) for s in range(3)])
    k = D.encode_k32(frames, 32, 0, B) if hasattr(D, "encode_k32") else None
    for f in range(3):
        if k is not None:
            assert np.array_equal(k[f], O.encode_frame_b(frames[f], B, 32, 0, k32=True))
        ku = D.encode(frames[f], 7, 0, block_size=B)
        assert np.array_equal(ku, O.encode_frame_b(frames[f], B, 7, 0))
    ku = D.encode(frames, 7, 0, block_size=B)
    for f in range(3):
        assert np.array_equal(ku[f], O.encode_frame_b(frames[f], B, 7, 0))
        assert np.array_equal(D.decode(ku[f], H, W, 7, 0, block_size=B),
                              O.decode_frame_b(ku[f], H, W, B, 7, 0))


# ---- Bluestein block sizes (vcf_pocketfft_blue.h): fftblue over cfftp ----

BLUE = json.load(open(os.path.join(GOLDEN, "manifest_blue.json")))


@pytest.mark.parametrize("case", BLUE["cases"], ids=lambda c: c["name"])
def test_bluestein_block_size_matches_reference_golden(case):
    """The reference's own encode_fn/decode_fn at -B 191 and -B 478 (2 x 239),
    lengths pocketfft plans with Bluestein (make_golden_blue.py), bit for bit."""
    d = np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))
    B, Q, flags = _qf(case["flags"])
    H, W = d["rgb"].shape[:2]
    k = D.encode(d["rgb"], Q, flags, block_size=B)
    assert np.array_equal(k, d["k"])
    assert np.array_equal(D.decode(d["k"], H, W, Q, flags, block_size=B), d["decoded"])


@pytest.mark.parametrize("B", [199, 223, 271, 389, 431, 509, 613])
@pytest.mark.parametrize("Q,flags", [(32, 0), (5, 3)])
def test_bluestein_block_size_vs_oracle(B, Q, flags):
    """Odd and even Bluestein lengths whose padded cfftp lengths use every
    pass (2, 3, 4, 5, 7, 8, 11), with -x and -p: kernels vs the oracle."""
    H, W = B + 2, B - 3
    rng = np.random.default_rng(B + Q)
    rgb = _smooth(H, W, B) if Q == 32 else rng.integers(0, 256, (H, W, 3), np.uint8)
    k = D.encode(rgb, Q, flags, block_size=B)
    assert np.array_equal(k, O.encode_frame_b(rgb, B, Q, flags))
    assert np.array_equal(D.decode(k, H, W, Q, flags, block_size=B), O.decode_frame_b(k, H, W, B, Q, flags))


@pytest.mark.parametrize("B", [1, 2, 3, 4, 7, 12, 16, 64, 130])
@pytest.mark.parametrize("flags", [2, 3])
def test_perceptual_any_block_size_vs_oracle(B, flags):
    """-p for B != 8 (2D-DCT.py:85-90, :313-327, :421-435) with the resized
    tables (cv2 restated, unpinned): kernels vs the oracle's pipeline."""
    H, W = B + 5, 2 * B + 3
    rgb = _smooth(H, W, B + flags)
    k = D.encode(rgb, 7, flags, block_size=B)
    assert np.array_equal(k, O.encode_frame_b(rgb, B, 7, flags))
    assert np.array_equal(D.decode(k, H, W, 7, flags, block_size=B), O.decode_frame_b(k, H, W, B, 7, flags))


def test_perceptual_b8_generic_kernel_equals_fused():
    """At B = 8 the resize is the identity: the generic kernels' -p equals the fused 8x8 kernels'."""
    import vcf_amd._lib as L
    from vcf_amd.device import DeviceBuffer
    rgb = _smooth(40, 56, 3)
    Hp, Wp = 40, 56
    for flags in (2, 3):
        fused = D.encode(rgb, 32, flags)
        din, dout = DeviceBuffer.from_array(rgb), DeviceBuffer(Hp * Wp * 3)
        L.call("vcf_dct_dz_encode_any", din.ptr, 1, 40, 56, 8, 32, flags, dout.ptr, None)
        anyk = dout.download(np.empty((Hp, Wp, 3), np.uint8))
        assert np.array_equal(anyk, fused)
        dec = DeviceBuffer(40 * 56 * 3)
        L.call("vcf_dct_dz_decode_any", dout.ptr, 1, 40, 56, 8, 32, flags, dec.ptr, None)
        assert np.array_equal(dec.download(np.empty((40, 56, 3), np.uint8)), D.decode(fused, 40, 56, 32, flags))
        for b in (din, dout, dec):
            b.free()
