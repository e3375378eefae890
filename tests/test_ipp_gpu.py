"""IPP temporal tools on the GPU (vcf_amd/csrc/vcf_ipp.hip through the C ABI)
against the reference's own block matching / compensation (tests/golden/
ipp.npz) and the oracle (oracle/vcf_ipp_oracle.c) on seeded inputs, plus the
IPP_DCT.py drop-in end to end: encode, decode, decode == encoder's loop."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN, ROOT
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _cases():
    with open(os.path.join(GOLDEN, "manifest_ipp.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLDEN, "ipp.npz"))


@pytest.fixture(scope="module")
def K():
    from vcf_amd import ipp
    return ipp


@pytest.mark.parametrize("fast", [False, True], ids=["full", "tss"])
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_block_matching_and_mc_match_reference(K, gold, case, fast):
    fr = gold[f"{case['name']}_frames"]
    tag = f"{case['name']}_{'fast' if fast else 'full'}"
    for t in range(1, case["n"]):
        mv = K.block_matching(fr[t - 1], fr[t], case["bs"], case["sr"], fast)
        assert np.array_equal(mv, gold[f"{tag}_mv"][t - 1]), f"frame {t}"
        comp = K.motion_compensate(fr[t - 1], mv, case["bs"])
        assert np.array_equal(comp, gold[f"{tag}_comp"][t - 1]), f"frame {t}"


def _moving(H, W, n, seed, noise=4):
    rng = np.random.Generator(np.random.PCG64(seed))
    base = rng.integers(0, 256, (H // 4 + 20, W // 4 + 20, 3)).astype(np.float64)
    base = np.kron(base, np.ones((4, 4, 1)))          # blocky texture, strong SAD minima
    out = []
    for t in range(n):
        dy, dx = (5 * t) % 23, (3 * t + t * t) % 29
        f = base[dy:dy + H, dx:dx + W] + rng.normal(0, noise, (H, W, 3))
        out.append(np.clip(np.rint(f), 0, 255).astype(np.uint8))
    return out


@pytest.mark.parametrize("H,W,bs,sr", [(64, 64, 16, 8), (96, 130, 16, 12), (77, 91, 8, 5), (128, 128, 32, 16),
                                       (40, 64, 4, 3), (16, 16, 16, 8), (64, 48, 64, 32), (33, 35, 7, 0),
                                       (61, 99, 12, 7), (80, 83, 20, 9), (50, 50, 16, 0), (90, 131, 4, 32)])
@pytest.mark.parametrize("fast", [False, True], ids=["full", "tss"])
def test_block_matching_vs_oracle(K, H, W, bs, sr, fast):
    fr = _moving(H, W, 3, H * W + bs)
    for t in (1, 2):
        mv = K.block_matching(fr[t - 1], fr[t], bs, sr, fast)
        assert np.array_equal(mv, O.ipp_block_matching(fr[t - 1], fr[t], bs, sr, fast))
        assert np.array_equal(K.motion_compensate(fr[t - 1], mv, bs), O.ipp_motion_compensate(fr[t - 1], mv, bs))


@pytest.mark.parametrize("bs,sr", [(16, 8), (8, 5), (12, 3), (32, 16), (4, 32)])
def test_full_search_word_and_byte_kernels_agree(K, bs, sr):
    """The word kernel (default for bs % 4 == 0) and the byte kernel give the
    same vectors, ties included (flat areas, textured areas, frame edges)."""
    rng = np.random.Generator(np.random.PCG64(bs * 100 + sr))
    fr = _moving(120, 200, 2, bs + sr)
    noisy = rng.integers(0, 256, (120, 200, 3), dtype=np.uint8)
    flat = np.full((120, 200, 3), 40, np.uint8)
    for a, b in ((fr[0], fr[1]), (noisy, fr[1]), (flat, flat), (fr[1], noisy)):
        try:
            K.set_full_search_variant(1)
            want = K.block_matching(a, b, bs, sr, False)
        finally:
            K.set_full_search_variant(0)
        assert np.array_equal(K.block_matching(a, b, bs, sr, False), want)


@pytest.mark.parametrize("sr", [8, 4, 16, 32, 1, 0])
def test_tss16_parallel_rounds_agree_with_serial_kernel(K, sr):
    """bs 16 --fast: the parallel-round kernel (default) and the serial one give
    the same vectors -- smooth motion, noise (centres that wander and leave
    the staged window), flat frames, frame edges."""
    rng = np.random.Generator(np.random.PCG64(sr + 7))
    fr = _moving(144, 208, 2, 5 + sr)
    noisy = rng.integers(0, 256, (144, 208, 3), dtype=np.uint8)
    flat = np.full((144, 208, 3), 90, np.uint8)
    for a, b in ((fr[0], fr[1]), (noisy, fr[1]), (fr[1], noisy), (flat, flat), (noisy, noisy[::-1].copy())):
        try:
            K.set_full_search_variant(1)
            want = K.block_matching(a, b, 16, sr, True)
        finally:
            K.set_full_search_variant(0)
        got = K.block_matching(a, b, 16, sr, True)
        assert np.array_equal(got, want)
        assert np.array_equal(got, O.ipp_block_matching(a, b, 16, sr, True))


def test_flat_frames_tie_break_first_minimum(K):
    """All SADs equal: the first in-bounds candidate (top-left of the window) wins (full), (0,0) for TSS."""
    f = np.full((64, 64, 3), 77, np.uint8)
    mv = K.block_matching(f, f, 16, 8, False)
    assert np.array_equal(mv, O.ipp_block_matching(f, f, 16, 8, False))
    assert tuple(mv[1, 1]) == (-8.0, -8.0) and tuple(mv[0, 0]) == (0.0, 0.0)
    assert not K.block_matching(f, f, 16, 8, True).any()


def test_frame_smaller_than_block(K):
    f = np.zeros((10, 12, 3), np.uint8)
    mv = K.block_matching(f, f, 16, 8, False)
    assert mv.shape == (0, 0, 2)
    assert not K.motion_compensate(f + 9, mv, 16).any()


def test_mc_out_of_bounds_and_fractional_vectors(K):
    rng = np.random.Generator(np.random.PCG64(3))
    f = rng.integers(0, 256, (48, 80, 3), dtype=np.uint8)
    mv = rng.uniform(-40, 40, (3, 5, 2)).astype(np.float32)    # many out of bounds, fractional -> int()
    assert np.array_equal(K.motion_compensate(f, mv, 16), O.ipp_motion_compensate(f, mv, 16))


def test_residual_and_reconstruct(K):
    rng = np.random.Generator(np.random.PCG64(4))
    a, b = rng.integers(0, 256, (2, 37, 53, 3), dtype=np.uint8)
    r = K.residual(a, b)
    assert np.array_equal(r, O.ipp_residual(a, b))
    assert np.array_equal(K.reconstruct(b, r), O.ipp_reconstruct(b, r))


def test_unsupported_sizes_raise(K):
    f = np.zeros((130, 130, 3), np.uint8)
    with pytest.raises(Exception):
        K.block_matching(f, f, 65, 8, False)
    with pytest.raises(Exception):
        K.block_matching(f, f, 16, 33, False)


def _write_seq(d, frames):
    for i, f in enumerate(frames):
        Image.fromarray(f).save(os.path.join(d, f"in_{i:04d}.png"))
    return os.path.join(d, "in_%04d.png")


def _ipp_loop(frames, gop, bs, sr, fast, Q):
    """The reference's temporal_filter (IPP_DCT.py:397-575, no RDO) over the oracle's
    2D-DCT round trip (the .tif is lossless, so encode_decode_proxy == oracle round trip)."""
    def rt(img):
        H, W = img.shape[:2]
        return O.decode_frame(O.encode_frame(img, Q), H, W, Q)
    recon, mvs = [], []
    for g0 in range(0, len(frames), gop):
        ref = rt(frames[g0])
        recon.append(ref)
        for p in range(1, min(gop, len(frames) - g0)):
            mv = O.ipp_block_matching(ref, frames[g0 + p], bs, sr, fast)
            comp = O.ipp_motion_compensate(ref, mv, bs)
            ref = O.ipp_reconstruct(comp, rt(O.ipp_residual(frames[g0 + p], comp)))
            recon.append(ref)
            mvs.append(mv)
    return recon, mvs


@pytest.mark.parametrize("fast", [False, True], ids=["full", "tss"])
def test_ipp_codec_encode_decode_matches_oracle_loop(tmp_path, fast):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.ipp import CoDec
    frames = _moving(72, 96, 7, 11)
    pat = _write_seq(str(tmp_path), frames)
    enc_prefix, dec_prefix = str(tmp_path / "enc" / "v"), str(tmp_path / "dec" / "v")
    flags = ["-N", "7", "-G", "3", "-M", "16", "-S", "8"] + (["--fast"] if fast else [])
    c = CoDec(P.parse(P.ipp_parser(), ["encode", "-i", pat, "-O", enc_prefix] + flags))
    total = c.encode()
    meta = json.load(open(enc_prefix + "_meta.json"))
    assert meta["n_frames"] == 7 and meta["gop_size"] == 3 and len(meta["I_info"]) == 3 and len(meta["P_info"]) == 4
    assert total == meta["total_bits"]
    for i in range(3):
        assert os.path.exists(f"{enc_prefix}_I_{i}_enc.tif") and os.path.exists(f"{enc_prefix}_I_{i}_enc_shape.bin")
    for i in range(4):
        assert os.path.exists(f"{enc_prefix}_P_{i}_enc.tif")
    assert os.path.exists(f"{enc_prefix}_O_0006.png")
    d = CoDec(P.parse(P.ipp_parser(), ["decode", "-i", enc_prefix, "-O", dec_prefix, "-M", "16"]))
    assert d.decode() == 7
    want, want_mv = _ipp_loop(frames, 3, 16, 8, fast, 32)
    with np.load(enc_prefix + "_mv.npz", allow_pickle=False) as z:
        assert np.array_equal(z["mv_f32"], np.stack(want_mv))
    for i in range(7):
        got = np.asarray(Image.open(f"{dec_prefix}_{i:04d}.png").convert("RGB"))
        assert np.array_equal(got, want[i]), f"frame {i}"


def test_ipp_cli(tmp_path):
    frames = _moving(48, 64, 4, 5)
    pat = _write_seq(str(tmp_path), frames)
    cli = os.path.join(ROOT, "vcf_amd", "cli", "IPP_DCT.py")
    enc, dec = str(tmp_path / "e"), str(tmp_path / "d")
    for argv in (["encode", "-i", pat, "-O", enc, "-N", "4", "-G", "2"], ["decode", "-i", enc, "-O", dec]):
        r = subprocess.run([sys.executable, cli] + argv, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
    assert all(os.path.exists(f"{dec}_{i:04d}.png") for i in range(4))


def test_ipp_over_2d_dwt_matches_oracle_loop(tmp_path):
    """--st 2D-DWT (IPP_DCT.py:45-87 subclasses the module --st names): I frames
    and residuals coded by the 2D-DWT codec (3l+1 subband TIFFs per frame); the
    decoded sequence equals the reference's GOP loop over the oracle's DWT
    round trip, and the CLI takes the DWT options."""
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.ipp import codec_class
    frames = _moving(64, 96, 5, 23)
    pat = _write_seq(str(tmp_path), frames)
    enc, dec = str(tmp_path / "enc" / "v"), str(tmp_path / "dec" / "v")
    p = P.ipp_parser(space_transform="2D-DWT")
    flags = ["--st", "2D-DWT", "-N", "5", "-G", "3", "-M", "16", "-S", "6", "-l", "3", "-w", "bior4.4", "-q", "16"]
    cls = codec_class("2D-DWT")
    cls(P.parse(p, ["encode", "-i", pat, "-O", enc] + flags)).encode()
    assert os.path.exists(f"{enc}_P_0_enc_LL_3.tif") and os.path.exists(f"{enc}_I_1_enc_HH_1.tif")
    d = cls(P.parse(p, ["decode", "-i", enc, "-O", dec, "-M", "16", "--st", "2D-DWT", "-l", "3", "-w", "bior4.4",
                        "-q", "16"]))
    assert d.decode() == 5

    def rt(img):
        H, W = img.shape[:2]
        return O.dwt_decode_frame(O.dwt_encode_frame(img, "bior4.4", 3, 16), H, W, "bior4.4", 3, 16)
    want = []
    for g0 in range(0, 5, 3):
        ref = rt(frames[g0])
        want.append(ref)
        for p_ in range(1, min(3, 5 - g0)):
            mv = O.ipp_block_matching(ref, frames[g0 + p_], 16, 6, False)
            comp = O.ipp_motion_compensate(ref, mv, 16)
            ref = O.ipp_reconstruct(comp, rt(O.ipp_residual(frames[g0 + p_], comp)))
            want.append(ref)
    for i in range(5):
        got = np.asarray(Image.open(f"{dec}_{i:04d}.png").convert("RGB"))
        assert np.array_equal(got, want[i]), f"frame {i}"
    cli = os.path.join(ROOT, "vcf_amd", "cli", "IPP_DCT.py")
    r = subprocess.run([sys.executable, cli, "encode", "-i", pat, "-O", str(tmp_path / "c" / "v")] + flags,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


def _ipp_loop_indices(frames, gop, bs, sr, fast, Q):
    """_ipp_loop's per-frame index arrays (what each frame's .tif holds) and motion fields."""
    ks, mvs = [], []
    for g0 in range(0, len(frames), gop):
        H, W = frames[g0].shape[:2]
        k = O.encode_frame(frames[g0], Q)
        ks.append(k)
        ref = O.decode_frame(k, H, W, Q)
        for p in range(1, min(gop, len(frames) - g0)):
            mv = O.ipp_block_matching(ref, frames[g0 + p], bs, sr, fast)
            comp = O.ipp_motion_compensate(ref, mv, bs)
            k = O.encode_frame(O.ipp_residual(frames[g0 + p], comp), Q)
            ks.append(k)
            ref = O.ipp_reconstruct(comp, O.decode_frame(k, H, W, Q))
            mvs.append(mv)
    return ks, mvs


@pytest.mark.parametrize("fast", [False, True], ids=["full", "tss"])
@pytest.mark.parametrize("n,gop,H,W", [(7, 3, 72, 96), (10, 4, 64, 80), (5, 10, 48, 64)])
def test_device_ipp_equals_reference_loop(n, gop, H, W, fast):
    """The HBM-resident C5 path (vcf_amd/codec/ipp_device.py: GOPs in lock step,
    batched DCT + GPU TIFF deflate): every gathered file equals the host TIFF
    writer's file of the reference loop's indices for that frame, and the motion
    fields are the reference loop's (IPP_DCT.py:397-575 restated by the oracle)."""
    from vcf_amd.codec.ipp_device import DeviceIPP
    from vcf_amd.codec.tiff import imread_bytes, imwrite_bytes
    from vcf_amd.device import DeviceBuffer
    frames = _moving(H, W, n, 17 + n)
    job = DeviceIPP(None, 0, 1, n, H, W, 32, gop, 16, 8, fast)
    stages = {}
    sizes, got, mvs = job.run(DeviceBuffer.from_array(np.stack(frames)), stages)
    ks, want_mv = _ipp_loop_indices(frames, gop, 16, 8, fast, 32)
    assert len(got) == n and len(mvs) == len(want_mv)
    for i in range(n):
        want = imwrite_bytes(ks[i])
        assert bytes(got[i]) == want and sizes[i] == len(want), i
        assert np.array_equal(imread_bytes(bytes(got[i])), ks[i])
    for a, b in zip(mvs, want_mv):
        assert np.array_equal(a, b)
    assert set(stages) >= {"gop_loop", "pack", "gatherv"}
