"""BASELINE.json's configs at their own sizes on the HIP path.

- C1 (512x512 RGB PNG, 2D-DCT B=8 + deadzone q=32 + TIFF; 2D-DCT.py:268-468):
  the drop-in CoDec's encode_fn/decode_fn on the two 512x512 cases the
  reference itself coded (tests/golden/manifest.json `big_cases`): SHA-256 of
  the indices, the .tif bytes and the decoded PNG's pixels equal the
  reference's.
- C4's per-rank batch (256 1080p frames over 8 ranks = 32 per launch) and the
  bench's 64 x 4K launch (1.59 GB in), and 96 x 4K (2.39 GB: frame offsets past 2^31 bytes): one launch
  each, frames first / middle / last against the oracle.
- C5 (IPP_DCT 4K; IPP_DCT.py:344-395): one 4K frame pair of full search and
  three-step search (bs 16, S 8), compensation, residual and reconstruction
  against the oracle; one GOP of the IPP CoDec at 4K against the reference's
  GOP loop (oracle-restated, tests/test_ipp_gpu.py::_ipp_loop).
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _synth():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.synth


@pytest.mark.parametrize("name", ["smooth_512x512", "rand_512x512"])
def test_c1_512_codec_matches_reference_hashes(tmp_path, manifest, name):
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    case = [c for c in manifest["big_cases"] if c["name"] == name][0]
    rgb = _synth()(case["kind"], case["H"], case["W"], case["seed"])
    assert _sha(rgb) == case["sha256"]["rgb"]
    src = str(tmp_path / "original.png")
    Image.fromarray(rgb).save(src)
    enc = CoDec(P.parse(P.dct_parser(), ["encode"]))
    nbytes = enc.encode_fn(src, str(tmp_path / "encoded"))
    tif = open(str(tmp_path / "encoded.tif"), "rb").read()
    assert nbytes == len(tif) == case["encode_bytes"]
    assert _sha(np.frombuffer(tif, np.uint8)) == case["sha256"]["tif"]
    assert _sha(np.asarray(enc.decompress(tif))) == case["sha256"]["k"]
    dec = CoDec(P.parse(P.dct_parser(), ["decode"]))
    dec.decode_fn(str(tmp_path / "encoded"), str(tmp_path / "decoded.png"))
    out = np.asarray(Image.open(str(tmp_path / "decoded.png")))
    assert _sha(out) == case["sha256"]["decoded"]


def _smooth(H, W, seed):
    from vcf_amd.synthetic import synth_frame
    return synth_frame(H, W, seed)


@pytest.mark.parametrize("H,W,n", [(1080, 1920, 32), (2160, 3840, 64), (2160, 3840, 96)],
                         ids=["c4_32x1080p", "bench_64x4k", "96x4k_past_2GiB"])
def test_full_size_single_launch_vs_oracle(H, W, n):
    import vcf_amd.dct as D
    from vcf_amd.device import DeviceBuffer, Stream
    pats = [_smooth(H, W, s) for s in range(3)]
    rng = np.random.default_rng(n)
    noise = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    fb = H * W * 3
    src = DeviceBuffer(n * fb)
    first, mid, last = 0, n // 2, n - 1
    chosen = {first: pats[0], mid: noise, last: pats[2]}
    s = Stream()
    for f in range(n):
        src.upload(chosen.get(f, pats[1]), stream=s, offset=f * fb)
    s.synchronize()
    dst = DeviceBuffer(n * fb)
    D.encode_device(src, n, H, W, 32, 0, out=dst, stream=s)
    s.synchronize()
    assert n < 96 or n * fb > (1 << 31)      # 96 x 4K: frame offsets past 2^31 bytes
    for f, rgb in chosen.items():
        got = dst.download(np.empty((H, W, 3), np.uint8), offset=f * fb)
        assert np.array_equal(got, O.encode_frame(rgb, 32, 0)), f"frame {f}"


def test_c5_4k_frame_pair_tools_vs_oracle():
    from test_ipp_gpu import _moving
    from vcf_amd import ipp as K
    ref, cur = _moving(2160, 3840, 2, 9)
    for fast in (False, True):
        mv = K.block_matching(ref, cur, 16, 8, fast)
        want = O.ipp_block_matching(ref, cur, 16, 8, fast)
        assert mv.shape == (135, 240, 2)
        assert np.array_equal(mv, want), "tss" if fast else "full"
    comp = K.motion_compensate(ref, mv, 16)
    assert np.array_equal(comp, O.ipp_motion_compensate(ref, mv, 16))
    res = K.residual(cur, comp)
    assert np.array_equal(res, O.ipp_residual(cur, comp))
    rec = O.decode_frame(O.encode_frame(res, 32), 2160, 3840, 32)
    assert np.array_equal(K.reconstruct(comp, rec), O.ipp_reconstruct(comp, rec))


def test_c5_4k_gop_codec_vs_reference_loop(tmp_path):
    from test_ipp_gpu import _ipp_loop, _moving, _write_seq
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.ipp import CoDec
    frames = _moving(2160, 3840, 3, 17)
    pat = _write_seq(str(tmp_path), frames)
    enc, dec = str(tmp_path / "enc" / "v"), str(tmp_path / "dec" / "v")
    c = CoDec(P.parse(P.ipp_parser(), ["encode", "-i", pat, "-O", enc, "-N", "3", "-G", "3", "-M", "16",
                                       "-S", "8"]))
    assert c.encode() > 0
    assert CoDec(P.parse(P.ipp_parser(), ["decode", "-i", enc, "-O", dec, "-M", "16"])).decode() == 3
    want, want_mv = _ipp_loop(frames, 3, 16, 8, False, 32)
    with np.load(enc + "_mv.npz", allow_pickle=False) as z:
        assert np.array_equal(z["mv_f32"], np.stack(want_mv))
    for i in range(3):
        got = np.asarray(Image.open(f"{dec}_{i:04d}.png").convert("RGB"))
        assert np.array_equal(got, want[i]), f"frame {i}"
