"""The opt-in lifting form of bior4.4 (vcf_dwt_dz_encode_lift / _decode_lift,
csrc/vcf_dwt_lift.h) against the bit-exact oracle: NOT bit-exact by design,
so the tolerance is written here -- every index and every decoded byte within
+-1, and on natural-image-like and noise frames (no values sitting on a
rounding boundary) at most 1e-4 of them off at all at Q = 32."""
import numpy as np
import pytest

from vcf_amd import synthetic as bench
from oracle import oracle as O

pytestmark = pytest.mark.gpu

INDEX_TOL = 1        # |k_lift - k_exact|
BYTE_TOL = 1         # |decoded_lift - decoded_exact|
RARE = 1e-4          # fraction allowed off on frames without exact ties
RARE_FINE = 1e-3     # the same on noise at fine steps (Q <= 32), any level count
# (at Q = 300 every detail index of a noise frame is 0 and the image is LL's
# smooth interpolation of multiples of 300, whose samples land on integers: up
# to 30 % of the bytes one off, 75.0000000000011 vs 74.9999999999999 -- only
# the +-1 bound holds there)


def _index_diff(ref, got):
    """(fraction of indices that differ, max |dk|) over a frame's subbands."""
    bad = tot = 0
    worst = 0
    for name, v in ref.items():
        a, b = v.astype(np.int64), got[name].astype(np.int64)
        d = a - b if name.startswith("LL") else (a - b + 128) % 256 - 128   # u8 indices wrap
        bad += int(np.count_nonzero(d))
        tot += d.size
        worst = max(worst, int(np.abs(d).max()))
    return bad / tot, worst


def _frames():
    rng = np.random.Generator(np.random.PCG64(7))
    flat = np.full((270, 480, 3), 100, np.uint8)
    flat[64:192, 100:300] = (30, 200, 90)
    return {
        "synthetic": (bench.synth_frame(270, 480, 3), True),
        "noise": (rng.integers(0, 256, (270, 480, 3), dtype=np.uint8), True),
        "odd_shape": (rng.integers(0, 256, (133, 251, 3), dtype=np.uint8), True),
        "flat_regions": (flat, False),
        "white": (np.full((270, 480, 3), 255, np.uint8), False),
        "ramp": (np.broadcast_to((np.arange(480) // 2 % 256).astype(np.uint8)[None, :, None],
                                 (270, 480, 3)).copy(), False),
    }


@pytest.mark.parametrize("name", list(_frames()))
def test_lift_encode_within_one_index(name):
    import vcf_amd.dwt as DW
    rgb, natural = _frames()[name]
    H, W = rgb.shape[:2]
    ref = O.dwt_encode_frame(rgb, "bior4.4", 5, 32)
    got = DW.encode(rgb, "bior4.4", 5, 32, lifting=True)[0]
    frac, worst = _index_diff(ref, got)
    assert worst <= INDEX_TOL, (name, worst)
    if natural:
        assert frac <= RARE, (name, frac)


@pytest.mark.parametrize("name", list(_frames()))
def test_lift_decode_within_one_byte(name):
    import vcf_amd.dwt as DW
    rgb, natural = _frames()[name]
    H, W = rgb.shape[:2]
    ref = O.dwt_encode_frame(rgb, "bior4.4", 5, 32)
    want = O.dwt_decode_frame(ref, H, W, "bior4.4", 5, 32)
    got = DW.decode(ref, H, W, "bior4.4", 5, 32, lifting=True)
    assert got.shape == want.shape
    d = np.abs(got.astype(np.int64) - want.astype(np.int64))
    assert d.max() <= BYTE_TOL, (name, int(d.max()))
    if natural:
        assert np.count_nonzero(d) / d.size <= RARE, name


@pytest.mark.parametrize("Q", [1, 7, 32, 300])
@pytest.mark.parametrize("L", [1, 2, 6])
def test_lift_levels_and_steps(L, Q):
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(L * 100 + Q))
    frames = rng.integers(0, 256, (2, 96, 130, 3), dtype=np.uint8)
    got = DW.encode(frames, "bior4.4", L, Q, lifting=True)
    for f in range(2):
        ref = O.dwt_encode_frame(frames[f], "bior4.4", L, Q)
        frac, worst = _index_diff(ref, got[f])
        assert worst <= INDEX_TOL and (Q > 32 or frac <= RARE_FINE), (f, frac, worst)
        want = O.dwt_decode_frame(ref, 96, 130, "bior4.4", L, Q)
        out = DW.decode(ref, 96, 130, "bior4.4", L, Q, lifting=True)
        d = np.abs(out.astype(np.int64) - want.astype(np.int64))
        assert d.max() <= BYTE_TOL, f
        assert Q > 32 or np.count_nonzero(d) / d.size <= RARE_FINE, (f, np.count_nonzero(d))


def test_lift_4k_batch_matches_product_path():
    """C3's frame size and batch shape: the lifting encode against the
    bit-exact product kernels (the oracle is too slow for 8 4K frames)."""
    import vcf_amd.dwt as DW
    frames = np.stack([bench.synth_frame(2160, 3840, 3 + f) for f in range(2)])
    exact = DW.encode(frames, "bior4.4", 5, 32)
    lift = DW.encode(frames, "bior4.4", 5, 32, lifting=True)
    for f in range(2):
        frac, worst = _index_diff(exact[f], lift[f])
        assert worst <= INDEX_TOL and frac <= RARE, (f, frac, worst)
    want = DW.decode(exact, 2160, 3840, "bior4.4", 5, 32)
    got = DW.decode(exact, 2160, 3840, "bior4.4", 5, 32, lifting=True)
    d = np.abs(got.astype(np.int64) - want.astype(np.int64))
    assert d.max() <= BYTE_TOL and np.count_nonzero(d) / d.size <= RARE


def test_lift_rejects_other_wavelets():
    import vcf_amd.dwt as DW
    with pytest.raises(ValueError):   # VCFInvalidArgument
        DW.encode(np.zeros((32, 32, 3), np.uint8), "db5", 2, 32, lifting=True)


def _unfused(fn):
    """fn() with the lifting path's level pairs unfused (one launch per level)."""
    from vcf_amd import _lib as Lb
    Lb.call("vcf_dwt_lift_set_fused", 0)
    try:
        return fn()
    finally:
        Lb.call("vcf_dwt_lift_set_fused", 1)


@pytest.mark.parametrize("H,W,L,Q", [(96, 240, 2, 32), (64, 480, 5, 32), (32, 176, 3, 7), (200, 496, 2, 300),
                                     (256, 512, 4, 32), (256, 512, 5, 7), (2160, 3840, 5, 32)])
def test_lift_fused_levels12_equal_unfused(monkeypatch, H, W, L, Q):
    """Levels 1 + 2 (and 3 + 4: (256, 512, 4 / 5), C3) in one launch
    (lift_fwd12_kernel: planes with w % 4 == 0, w / 2 % 8 == 0, h % 4 == 0)
    compute the same operations as the level launches: identical bytes, one
    strip and several, partial last strips, the pair's LL as the last level
    (u16) and as float64 for the next."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H + W + L))
    frames = (np.stack([bench.synth_frame(H, W, 5), rng.integers(0, 256, (H, W, 3), dtype=np.uint8)])
              if H * W < 4e6 else bench.synth_frame(H, W, 5)[None])
    fused = DW.encode(frames, "bior4.4", L, Q, lifting=True)
    split = _unfused(lambda: DW.encode(frames, "bior4.4", L, Q, lifting=True))
    for f in range(len(frames)):
        for name in fused[f]:
            assert np.array_equal(fused[f][name], split[f][name]), (f, name)
    if H * W < 4e6:
        ref = O.dwt_encode_frame(frames[0], "bior4.4", L, Q)
        frac, worst = _index_diff(ref, fused[0])
        assert worst <= INDEX_TOL and frac <= RARE_FINE, (frac, worst)


@pytest.mark.parametrize("H,W,L,Q", [(96, 240, 2, 32), (64, 480, 5, 32), (32, 176, 3, 7), (200, 496, 2, 300),
                                     (256, 512, 4, 32), (256, 512, 5, 7), (2160, 3840, 5, 32)])
def test_lift_fused_levels21_decode_equal_unfused(monkeypatch, H, W, L, Q):
    """Inverse levels 2 + 1 in one launch (lift_inv21_kernel) against the two
    level launches: identical RGB bytes."""
    import vcf_amd.dwt as DW
    rng = np.random.Generator(np.random.PCG64(H * W + L))
    frames = (np.stack([bench.synth_frame(H, W, 6), rng.integers(0, 256, (H, W, 3), dtype=np.uint8)])
              if H * W < 4e6 else bench.synth_frame(H, W, 6)[None])
    sb = DW.encode(frames, "bior4.4", L, Q)
    fused = DW.decode(sb, H, W, "bior4.4", L, Q, lifting=True)
    split = _unfused(lambda: DW.decode(sb, H, W, "bior4.4", L, Q, lifting=True))
    assert np.array_equal(fused, split)
    if H * W < 4e6:
        want = O.dwt_decode_frame(sb[0], H, W, "bior4.4", L, Q)
        d = np.abs(fused[0].astype(np.int64) - want.astype(np.int64))
        assert d.max() <= BYTE_TOL   # (a small smooth frame at l = 2 lands on ties often: 1.3 % here)


# The north star's unit for the float DWT is the ULP (float64).  The lifting
# form computes other roundings than pywt's convolution (and its constants
# are the CDF 9/7 factorisation's, not pywt's tap values), so it is NOT
# within 1 ULP.  Measured (scripts/lift_tolerance.py on MI355X,
# profiles/r06_lift_tolerance.json): up to 3.1e7 ULP (p99
# 3.1e6) over coefficients with |pywt| >= 1, at most 8.2e-9 absolute on any
# coefficient, 1.7e-10 of the subband's largest magnitude on the 4K frame.
# These bounds (about 2x the measurement) are what the test holds it to.
LIFT_ULP_MAX = 1 << 26          # over coefficients with |pywt| >= 1
LIFT_ABS_MAX = 2e-8             # any coefficient, absolute


@pytest.mark.parametrize("name", ["synthetic", "noise", "odd_shape", "white", "uhd"])
def test_lift_float64_coefficients_vs_pywt(name):
    """The lifting path's float64 coefficients before quantization (every
    level, all three YCoCg channels) against pywt's restated by the oracle."""
    import vcf_amd.dwt as DW
    from oracle import lift_tolerance as LT
    if name == "uhd":
        rgb = bench.synth_frame(2160, 3840, 9)
    else:
        rgb = _frames()[name][0]
    got = DW.lift_coefficients(rgb, 5)
    r = LT.compare(got, rgb, 5)
    assert r["abs_max"] <= LIFT_ABS_MAX, r
    assert r["ulp_max"] <= LIFT_ULP_MAX, r
