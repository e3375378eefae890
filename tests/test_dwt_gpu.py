"""2D-DWT + deadzone on the GPU against the reference's files (tests/golden/
dwt_*.npz, made by src/2D-DWT.py) and the oracle, bit for bit."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu
_MAN = json.load(open(os.path.join(GOLDEN, "manifest_dwt.json")))
_SHORT = json.load(open(os.path.join(GOLDEN, "manifest_dwt_short.json")))


def _params(case):
    fl = case["flags"]
    w = fl[fl.index("-w") + 1] if "-w" in fl else "db5"
    Q = int(fl[fl.index("-q") + 1]) if "-q" in fl else 32
    return w, case["levels"], Q


@pytest.mark.parametrize("case", _MAN["cases"], ids=lambda c: c["name"])
def test_dwt_encode_decode_vs_reference(case):
    import vcf_amd.dwt as DW
    d = np.load(os.path.join(GOLDEN, f"dwt_{case['name']}.npz"))
    w, L, Q = _params(case)
    sb = DW.encode(d["rgb"], w, L, Q)[0]
    for name in case["subbands"]:
        assert np.array_equal(sb[name], d[name]), name
    out = DW.decode({n: d[n] for n in case["subbands"]}, case["H"], case["W"], w, L, Q)
    assert np.array_equal(out, d["decoded"])


@pytest.mark.parametrize("case", _SHORT["cases"], ids=lambda c: c["name"])
def test_dwt_short_subbands_vs_reference(case):
    """Frames whose last levels' subbands are shorter than F/2 (pywt's short-input
    branch in the inverse) against the reference's own files and decoded frame."""
    import vcf_amd.dwt as DW
    d = np.load(os.path.join(GOLDEN, case["file"]))
    w, L, Q = _params(case)
    sb = DW.encode(d["rgb"], w, L, Q)[0]
    for name in case["subbands"]:
        assert np.array_equal(sb[name], d[name]), name
    for variant in (0, 2):
        out = DW.decode({n: d[n] for n in case["subbands"]}, case["H"], case["W"], w, L, Q, variant=variant)
        assert np.array_equal(out, d["decoded"]), variant


@pytest.mark.parametrize("wavelet", ["db5", "bior4.4", "db10", "sym8", "coif5", "rbio3.9", "db20"])
@pytest.mark.parametrize("H,W,L", [(5, 7, 3), (23, 2, 2), (1, 1, 4), (40, 9, 5), (3, 64, 6)])
def test_dwt_short_lines_vs_oracle(wavelet, H, W, L):
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H * 131 + W * 7 + L))
    frames = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    got = DW.encode(frames, wavelet, L, 5, variant=2)
    out = DW.decode(got, H, W, wavelet, L, 5)
    for f in range(2):
        ref = O.dwt_encode_frame(frames[f], wavelet, L, 5)
        for name, arr in ref.items():
            assert np.array_equal(got[f][name], arr), (f, name)
        assert np.array_equal(out[f], O.dwt_decode_frame(got[f], H, W, wavelet, L, 5))


@pytest.mark.parametrize("variant", [0, 1, 2, 6, 20], ids=["default", "fused", "separable", "strip", "hybrid"])
@pytest.mark.parametrize("wavelet", ["db5", "bior4.4", "haar", "sym4", "coif2", "db9", "db10"])
@pytest.mark.parametrize("H,W,L,Q", [(96, 128, 3, 32), (67, 45, 2, 7), (256, 160, 5, 16), (8, 10, 1, 1),
                                     (141, 301, 4, 3), (17, 200, 3, 32)])
def test_dwt_vs_oracle(wavelet, H, W, L, Q, variant):
    import vcf_amd.dwt as DW
    shapes = O.dwt_shapes(H, W, L)
    rng = np.random.Generator(np.random.PCG64(H * W + L))
    frames = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    if variant in (1, 6) and wavelet == "db10":      # 20 taps: the fused tile exceeds 64 KB of LDS
        with pytest.raises(NotImplementedError):
            DW.encode(frames, wavelet, L, Q, variant=1)
        return
    got = DW.encode(frames, wavelet, L, Q, variant=variant)
    for f in range(2):
        ref = O.dwt_encode_frame(frames[f], wavelet, L, Q)
        for name, arr in ref.items():
            assert np.array_equal(got[f][name], arr), (f, name)
    half = O.lib().vcfo_wavelet_len(O.wavelet_index(wavelet)) // 2
    dec_variant = {6: 1, 20: 0}.get(variant, variant)
    if min(shapes[-1]) < half:
        # pywt's short-input branch: the separable kernels (automatic choice) run it,
        # an explicit request for the fused tiles is refused
        if dec_variant == 1:
            with pytest.raises(NotImplementedError):
                DW.decode(got[0], H, W, wavelet, L, Q, variant=1)
        dec_variant = 0
    out = DW.decode(got, H, W, wavelet, L, Q, variant=dec_variant)
    for f in range(2):
        assert np.array_equal(out[f], O.dwt_decode_frame(got[f], H, W, wavelet, L, Q))


@pytest.mark.parametrize("wavelet", ["bior4.4", "db5"])
def test_dwt_4k_fused_equals_separable_and_oracle(wavelet):
    """Config C3 size: the fused and separable kernels agree on whole 4K frames, and frame 0 equals the oracle."""
    import vcf_amd.dwt as DW
    H, W, L, Q = 2160, 3840, 5, 32
    y, x = np.mgrid[0:H, 0:W]
    base = np.stack([128 + 60 * np.sin(x / 97 + c) + 50 * np.cos(y / 61 - c) for c in range(3)], -1)
    rng = np.random.Generator(np.random.PCG64(5))
    frames = np.stack([np.clip(base + rng.normal(0, 4, base.shape), 0, 255).astype(np.uint8) for _ in range(2)])
    a = DW.encode(frames, wavelet, L, Q, variant=1)
    b = DW.encode(frames, wavelet, L, Q, variant=2)
    c = DW.encode(frames, wavelet, L, Q, variant=3)   # the earlier three-barrier schedule of the fused kernels
    e = DW.encode(frames, wavelet, L, Q, variant=4)   # run-time taps
    f = DW.encode(frames, wavelet, L, Q, variant=5)   # level 1 staged as float
    g = DW.encode(frames, wavelet, L, Q, variant=6)   # strip kernels (sums started by their first product)
    h = DW.encode(frames, wavelet, L, Q, variant=7)   # strip kernels, sums started at 0.0
    ref = O.dwt_encode_frame(frames[0], wavelet, L, Q)
    for name in ref:
        assert np.array_equal(a[0][name], ref[name]), name
        assert np.array_equal(a[1][name], b[1][name]), name
        assert np.array_equal(c[1][name], a[1][name]), name
        assert np.array_equal(e[1][name], a[1][name]), name
        assert np.array_equal(f[1][name], a[1][name]), name
        assert np.array_equal(g[0][name], ref[name]), name
        assert np.array_equal(g[1][name], a[1][name]), name
        assert np.array_equal(h[1][name], a[1][name]), name
    da = DW.decode(a, H, W, wavelet, L, Q, variant=1)
    db = DW.decode(a, H, W, wavelet, L, Q, variant=2)
    assert np.array_equal(da, db)
    assert np.array_equal(DW.decode(a, H, W, wavelet, L, Q, variant=4), da)   # run-time taps
    assert np.array_equal(DW.decode(a, H, W, wavelet, L, Q, variant=5), da)   # no staging priority
    assert np.array_equal(da[0], O.dwt_decode_frame(a[0], H, W, wavelet, L, Q))
    assert np.abs(da.astype(int) - frames.astype(int)).mean() < 8     # a sane reconstruction


@pytest.mark.parametrize("wavelet", ["bior4.4", "db5"])
def test_dwt_4k_frame_pipeline(wavelet):
    """Frame chunks on the library's streams (encode variants 0/13-26, decode 0/6-11) give the bytes of the
    single-stream chain (encode 17, decode 9) on an odd batch of 4K frames; the last frame equals the oracle."""
    import vcf_amd.dwt as DW
    H, W, L, Q = 2160, 3840, 5, 32
    rng = np.random.Generator(np.random.PCG64(11))
    frames = rng.integers(0, 256, (5, H, W, 3), dtype=np.uint8)
    ref = DW.encode(frames, wavelet, L, Q, variant=17)
    for v in (0, 13, 14, 15, 16, 18, 19, 20, 21, 22, 23, 24, 25, 26):
        got = DW.encode(frames, wavelet, L, Q, variant=v)
        for f in range(5):
            for name in ref[f]:
                assert np.array_equal(got[f][name], ref[f][name]), (v, f, name)
    oref = O.dwt_encode_frame(frames[4], wavelet, L, Q)
    for name in oref:
        assert np.array_equal(ref[4][name], oref[name]), name
    dref = DW.decode(ref, H, W, wavelet, L, Q, variant=9)
    for v in (0, 6, 7, 8, 10, 11, 12, 13, 14, 15, 16):
        assert np.array_equal(DW.decode(ref, H, W, wavelet, L, Q, variant=v), dref), v
    assert np.array_equal(dref[4], O.dwt_decode_frame(ref[4], H, W, wavelet, L, Q))


@pytest.mark.parametrize("H,W,L,Q", [(67, 45, 2, 7), (141, 301, 4, 3)])
def test_dwt_frame_pipeline_small(H, W, L, Q):
    """The forced pipeline variants on small odd frames (the default keeps them on the caller's stream)."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H + W))
    frames = rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8)
    for wavelet in ("bior4.4", "sym4"):
        ref = DW.encode(frames, wavelet, L, Q, variant=0)
        for v in (13, 14, 16, 19, 20, 22, 23, 24, 25, 26):
            got = DW.encode(frames, wavelet, L, Q, variant=v)
            for f in range(3):
                for name in ref[f]:
                    assert np.array_equal(got[f][name], ref[f][name]), (wavelet, v, f, name)
        dref = DW.decode(ref, H, W, wavelet, L, Q, variant=0)
        for v in (6, 7, 10, 12, 14, 15, 16):   # 15 / 16: 32 x 32 / 128 x 8 inverse tiles (bior4.4)
            assert np.array_equal(DW.decode(ref, H, W, wavelet, L, Q, variant=v), dref), (wavelet, v)


def test_dwt_unknown_variant():
    import vcf_amd.dwt as DW
    with pytest.raises(ValueError):
        DW.encode(np.zeros((16, 16, 3), np.uint8), "db5", 2, 32, variant=28)
    with pytest.raises(ValueError):
        DW.decode(DW.encode(np.zeros((16, 16, 3), np.uint8), "db5", 2, 32), 16, 16, "db5", 2, 32, variant=19)


def test_dwt_errors():
    import vcf_amd.dwt as DW
    with pytest.raises(ValueError):
        DW.wavelet_index("nope")
    with pytest.raises(ValueError):
        DW.encode(np.zeros((8, 8, 3), np.uint8), "db5", 0, 32)


@pytest.mark.parametrize("case", _MAN["cases"][:5], ids=lambda c: c["name"])
def test_dwt_codec_files(tmp_path, case):
    """encode_fn writes the reference's subband files; decode_fn of the
    reference's files gives its decoded frame."""
    from PIL import Image
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dwt2d import CoDec
    from vcf_amd.codec.tiff import imread_bytes, imwrite_bytes
    d = np.load(os.path.join(GOLDEN, f"dwt_{case['name']}.npz"))
    src = str(tmp_path / "in.png")
    Image.fromarray(d["rgb"]).save(src)
    enc = str(tmp_path / "enc")
    c = CoDec(P.parse(P.dwt_parser(), ["encode"] + case["flags"]))
    n = c.encode_fn(src, enc)
    assert n == case["encode_bytes"]
    L = case["levels"]
    assert open(f"{enc}_LL_{L}.tif", "rb").read() == bytes(d["tif_LL"])
    for name in case["subbands"]:
        assert np.array_equal(imread_bytes(open(f"{enc}_{name}.tif", "rb").read()), d[name]), name
    ref = str(tmp_path / "ref")
    for name in case["subbands"]:
        with open(f"{ref}_{name}.tif", "wb") as f:
            f.write(imwrite_bytes(d[name]))
    out = str(tmp_path / "out.png")
    CoDec(P.parse(P.dwt_parser(), ["decode"] + case["flags"])).decode_fn(ref, out)
    assert np.array_equal(np.asarray(Image.open(out)), d["decoded"])


def test_cli_2d_dwt(tmp_path):
    import subprocess
    import sys
    from PIL import Image
    from conftest import ROOT
    rgb = np.random.Generator(np.random.PCG64(3)).integers(0, 256, (48, 64, 3), dtype=np.uint8)
    src, enc, dec = str(tmp_path / "o.png"), str(tmp_path / "e"), str(tmp_path / "d.png")
    Image.fromarray(rgb).save(src)
    for argv in (["encode", "-l", "2", "-w", "bior4.4", "-o", src, "-e", enc],
                 ["decode", "-l", "2", "-w", "bior4.4", "-e", enc, "-d", dec]):
        r = subprocess.run([sys.executable, "vcf_amd/cli/2D-DWT.py"] + argv, cwd=ROOT, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
    sb = O.dwt_encode_frame(rgb, "bior4.4", 2, 32)
    assert np.array_equal(np.asarray(Image.open(dec)), O.dwt_decode_frame(sb, 48, 64, "bior4.4", 2, 32))


@pytest.mark.parametrize("wavelet", ["bior4.4", "db5"])
@pytest.mark.parametrize("H,W,L,Q", [(64, 512, 2, 32), (128, 1024, 3, 7), (200, 600, 4, 16), (68, 516, 5, 1),
                                     (96, 1000, 2, 3), (264, 728, 5, 64)])
def test_dwt_band12_vs_oracle(wavelet, H, W, L, Q):
    """The fused level-1+2 band kernel (the default for bior4.4 / db5 on planes
    with h % 4 == 0, w % 4 == 0, at least 64 x 512): every subband equals the
    oracle and the level-by-level kernels (variant 27), whatever the band and
    tile cuts (partial last tile, one-row bands, wrapped halos)."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H * 7 + W + L))
    frames = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    frames[1] = np.clip(frames[1] // 8 + 100 + (np.arange(W)[None, :, None] // 3), 0, 255)   # smooth-ish
    got = DW.encode(frames, wavelet, L, Q)
    ref_chain = DW.encode(frames, wavelet, L, Q, variant=27)
    for f in range(2):
        ref = O.dwt_encode_frame(frames[f], wavelet, L, Q)
        for name, arr in ref.items():
            assert np.array_equal(got[f][name], arr), (f, name)
            assert np.array_equal(ref_chain[f][name], arr), (f, name)


@pytest.mark.parametrize("n", [1, 3, 8])
def test_dwt_band12_batches(n):
    """Batches of 1080p frames (the band count follows the batch) equal the level-by-level chain."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(n))
    frames = rng.integers(0, 256, (n, 1080, 1920, 3), dtype=np.uint8)
    a = DW.encode(frames, "bior4.4", 5, 32)
    b = DW.encode(frames, "bior4.4", 5, 32, variant=27)
    for f in range(n):
        for name in a[f]:
            assert np.array_equal(a[f][name], b[f][name]), (f, name)
    ref = O.dwt_encode_frame(frames[-1], "bior4.4", 5, 32)
    for name, arr in ref.items():
        assert np.array_equal(a[-1][name], arr), name


@pytest.mark.parametrize("wavelet", ["bior4.4", "db5"])
@pytest.mark.parametrize("H,W,L,Q", [(96, 128, 3, 32), (67, 45, 2, 7), (141, 301, 4, 3), (300, 530, 3, 16),
                                     (20, 1030, 2, 1), (44, 44, 3, 5)])
def test_dwt_line_decode_vs_oracle(wavelet, H, W, L, Q):
    """The line-based inverse levels (decode variant 0; 18 = level 1 only) against the tiled level kernels
    (variant 17) and the oracle: partial column tiles, odd subband sizes, the packed-LL coarsest level."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H * 7 + W + L))
    frames = rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8)
    got = DW.encode(frames, wavelet, L, Q)
    out = DW.decode(got, H, W, wavelet, L, Q)
    assert np.array_equal(out, DW.decode(got, H, W, wavelet, L, Q, variant=17))
    assert np.array_equal(out, DW.decode(got, H, W, wavelet, L, Q, variant=18))
    for f in (0, 2):
        assert np.array_equal(out[f], O.dwt_decode_frame(got[f], H, W, wavelet, L, Q))


@pytest.mark.parametrize("wavelet", ["bior4.4", "db5"])
def test_dwt_line_decode_4k(wavelet):
    """Config C3 frames: the line-based inverse equals the tiled level kernels and the oracle."""
    import vcf_amd.dwt as DW
    H, W, L, Q = 2160, 3840, 5, 32
    rng = np.random.Generator(np.random.PCG64(12))
    frames = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    got = DW.encode(frames, wavelet, L, Q)
    out = DW.decode(got, H, W, wavelet, L, Q)
    assert np.array_equal(out, DW.decode(got, H, W, wavelet, L, Q, variant=17))
    assert np.array_equal(out[1], O.dwt_decode_frame(got[1], H, W, wavelet, L, Q))


def _decode_unfused(DW, *a):
    """DW.decode with the inverse levels 2 + 1 as two line-kernel launches."""
    from vcf_amd import _lib as Lb
    Lb.call("vcf_dwt_set_inverse_band21", 0)
    try:
        return DW.decode(*a)
    finally:
        Lb.call("vcf_dwt_set_inverse_band21", 1)


@pytest.mark.parametrize("wavelet,H,W,L,Q", [
    ("bior4.4", 2160, 3840, 5, 32),      # C3
    ("db5", 2160, 3840, 5, 32),
    ("bior4.4", 96, 136, 2, 32),          # LL2 from the packed u16 subband; a partial last tile
    ("bior4.4", 120, 248, 3, 7),          # non-power-of-two Q
    ("db5", 200, 480, 4, 300),            # Q > 256: the int16 dequant
    ("bior4.4", 40, 40, 2, 1),            # subbands of 10 x 10: one tile, one band
    ("bior4.4", 44, 60, 3, 32),           # h1 = 22 = 2 h2, w1 = 30 = 2 h2: level 2 of 11 x 15
    ("bior4.4", 90, 140, 3, 32),          # h1 = 45 odd: the two launches (not halving evenly)
])
def test_dwt_decode_band21_equals_two_launches(wavelet, H, W, L, Q):
    """The inverse levels 2 + 1 in one launch (idwt_band21_kernel, LL1 on chip)
    give the bytes of the two line-kernel launches and of the oracle."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H * W + L))
    frames = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    frames[1] = np.broadcast_to(np.arange(W, dtype=np.uint8)[None, :, None], (H, W, 3))
    sb = DW.encode(frames, wavelet, L, Q)
    fused = DW.decode(sb, H, W, wavelet, L, Q)
    two = _decode_unfused(DW, sb, H, W, wavelet, L, Q)
    assert np.array_equal(fused, two)
    f = 1 if H * W > 1e6 else 0
    assert np.array_equal(fused[f], O.dwt_decode_frame(sb[f], H, W, wavelet, L, Q))
