"""GPU parity of the fused DCT+deadzone kernels (through the C ABI).

Bit-exact against (1) the golden vectors produced by the reference's own
glue (tests/golden, make_golden.py) and (2) the C oracle on seeded inputs,
including padding, -x, -p, non-power-of-two and wrapping quantization steps,
batched frames and full 4K/1080p frames.
"""
import numpy as np
import pytest

from conftest import case_params, golden_cases, load_case
from oracle import oracle as O

pytestmark = pytest.mark.gpu

D = pytest.importorskip("vcf_amd.dct")


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_encode_matches_reference_golden(case):
    z = load_case(case)
    Q, flags = case_params(case)
    k = D.encode(z["rgb"], Q, flags)
    assert k.shape == z["k"].shape
    assert np.array_equal(k, z["k"])


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_decode_matches_reference_golden(case):
    z = load_case(case)
    Q, flags = case_params(case)
    out = D.decode(z["k"], case["H"], case["W"], Q, flags)
    assert np.array_equal(out, z["decoded"])


def _rand(shape, seed, kind="rand"):
    rng = np.random.Generator(np.random.PCG64(seed))
    if kind == "rand":
        return rng.integers(0, 256, shape, dtype=np.uint8)
    if kind == "flat":
        H, W, _ = shape
        b = rng.integers(0, 256, ((H + 7) // 8, (W + 7) // 8, 3), dtype=np.uint8)
        return np.repeat(np.repeat(b, 8, 0), 8, 1)[:H, :W].copy()
    y, x = np.mgrid[0:shape[0], 0:shape[1]]
    v = np.stack([128 + 100 * np.sin(x / 13 + c) * np.cos(y / 7 - c) for c in range(3)], -1)
    v = v + rng.normal(0, 6, shape)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


SHAPES = [(8, 8), (16, 2048), (24, 4104), (72, 136), (13, 29), (100, 100), (9, 4097), (264, 320)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("Q,flags", [(32, 0), (7, 0), (1, 0), (32, 1), (32, 2), (5, 3), (64, 2)])
def test_encode_decode_vs_oracle(shape, Q, flags):
    H, W = shape
    rgb = _rand((H, W, 3), seed=H * 7919 + W + Q, kind="smooth" if H % 2 else "rand")
    k = D.encode(rgb, Q, flags)
    assert np.array_equal(k, O.encode_frame(rgb, Q, flags))
    out = D.decode(k, H, W, Q, flags)
    assert np.array_equal(out, O.decode_frame(k, H, W, Q, flags))


def test_flat_blocks_boundary_hazard():
    """Constant 8x8 blocks: the fp32 DC sits on k boundaries."""
    rgb = _rand((256, 512, 3), 3, "flat")
    for Q in (1, 2, 4, 8, 16, 32):
        assert np.array_equal(D.encode(rgb, Q), O.encode_frame(rgb, Q))


def test_batched_frames_equal_single():
    frames = np.stack([_rand((64, 96, 3), s) for s in range(5)])
    k = D.encode(frames, 32)
    for i in range(5):
        assert np.array_equal(k[i], O.encode_frame(frames[i], 32))
    out = D.decode(k, 64, 96, 32)
    for i in range(5):
        assert np.array_equal(out[i], O.decode_frame(k[i], 64, 96, 32))


def test_extreme_wrap_q1():
    """q=1: |k| > 127 wraps modulo 256 exactly like astype(uint8)."""
    rgb = (np.indices((64, 64)).sum(0) % 2 * 255).astype(np.uint8)[..., None].repeat(3, 2)
    k = D.encode(rgb, 1)
    assert np.array_equal(k, O.encode_frame(rgb, 1))
    assert np.array_equal(D.decode(k, 64, 64, 1), O.decode_frame(k, 64, 64, 1))


@pytest.mark.parametrize("shape", [(1080, 1920), (2160, 3840)])
def test_full_size_frames(shape):
    H, W = shape
    rgb = _rand((H, W, 3), 11, "smooth")
    k = D.encode(rgb, 32)
    assert np.array_equal(k, O.encode_frame(rgb, 32))
    out = D.decode(k, H, W, 32)
    assert np.array_equal(out, O.decode_frame(k, H, W, 32))


def test_zero_frames_and_errors():
    from vcf_amd.device import DeviceBuffer
    buf = DeviceBuffer(64)
    D.encode_device(buf, 0, 8, 8, out=DeviceBuffer(64))   # no-op
    with pytest.raises(ValueError):
        D.encode(np.zeros((8, 8), np.uint8))
    with pytest.raises(NotImplementedError):
        D.encode(np.zeros((16, 16, 3), np.uint8), 32, block_size=4097)   # beyond the run-time path
    with pytest.raises(ValueError):
        D.decode(np.zeros((8, 8, 3), np.uint8), 8, 8, 40000)


@pytest.mark.parametrize("variant", [0, 1, 3, 5])
@pytest.mark.parametrize("Q,flags", [(32, 0), (7, 0), (1, 0), (32, 1), (5, 3), (64, 2)])
def test_encode_variants_vs_oracle(variant, Q, flags):
    """Both encode kernels on shapes both support (no padding, W % 32 == 0)."""
    for H, W in [(8, 32), (64, 128), (40, 96), (136, 2048)]:
        rgb = _rand((H, W, 3), seed=H + W + Q, kind="rand" if W % 64 else "smooth")
        k = D.encode(rgb, Q, flags, variant=variant)
        assert np.array_equal(k, O.encode_frame(rgb, Q, flags)), (H, W)
    frames = np.stack([_rand((24, 160, 3), s) for s in range(7)])
    k = D.encode(frames, Q, flags, variant=variant)
    for i in range(7):
        assert np.array_equal(k[i], O.encode_frame(frames[i], Q, flags))


@pytest.mark.parametrize("Q", [1, 32, 256])
def test_encode_variant4_generic_colour(Q):
    """The A/B reference kernel (generic colour code) equals the oracle too."""
    for H, W in [(8, 32), (64, 128), (136, 2048)]:
        rgb = _rand((H, W, 3), seed=H * W + Q)
        assert np.array_equal(D.encode(rgb, Q, 0, variant=4), O.encode_frame(rgb, Q, 0)), (H, W)


def test_unknown_variant_rejected():
    with pytest.raises(ValueError):
        D.encode(np.zeros((16, 16, 3), np.uint8), 32, variant=99)


@pytest.mark.parametrize("shape", SHAPES + [(2160, 3840), (1080, 1920)])
@pytest.mark.parametrize("Q,flags", [(32, 0), (7, 1), (1, 0), (5, 3), (64, 2), (30001, 0)])
def test_decode_variants_vs_oracle(shape, Q, flags):
    """The decode kernels (0 automatic: column-per-lane with the dequantization
    table, 1 lane-per-block, 2 column-per-lane with the 32-bit multiply) are bit-exact."""
    H, W = shape
    rgb = _rand((H, W, 3), seed=H * 31 + W + Q, kind="smooth" if W % 2 else "rand")
    k = O.encode_frame(rgb, Q, flags) if H * W <= 1 << 20 else D.encode(rgb, Q, flags)
    want = O.decode_frame(k, H, W, Q, flags)
    for v in (0, 1, 2):
        assert np.array_equal(D.decode(k, H, W, Q, flags, variant=v), want), v


def test_decode_variants_batched():
    frames = np.stack([_rand((72, 4104, 3), seed=s, kind="smooth") for s in range(3)])
    k = D.encode(frames, 32, 0)
    a = D.decode(k, 72, 4104, 32, 0, variant=1)
    b = D.decode(k, 72, 4104, 32, 0, variant=2)
    for v in (0, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13):   # the default and the A/B variants of 2
        assert np.array_equal(D.decode(k, 72, 4104, 32, 0, variant=v), b), v
    assert np.array_equal(a, b)
    assert np.array_equal(a[2], O.decode_frame(k[2], 72, 4104, 32, 0))


@pytest.mark.parametrize("variant", [0, 1, 5])
@pytest.mark.parametrize("shape,n,flags", [((1080, 1920), 8, 0), ((100, 300), 400, 0), ((100, 300), 400, 1),
                                           ((72, 4104), 12, 0), ((13, 29), 900, 1)])
def test_packed_encode_batches(variant, shape, n, flags):
    """The tile kernels (scalar and packed-fp32 transforms, full-tile and
    generic copy-out) on large batches with partial last tiles, padding and
    both output layouts: equal to each other and spot-checked against the oracle."""
    H, W = shape
    rng = np.random.default_rng(H + W + n)
    frames = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    frames[: n // 2] = _rand((H, W, 3), 5, "smooth")
    want = D.encode(frames, 32, flags, variant=3)   # the column-per-lane kernel, independent code
    got = D.encode(frames, 32, flags, variant=variant)
    assert np.array_equal(got, want)
    for i in (0, n // 2, n - 1):
        assert np.array_equal(got[i], O.encode_frame(frames[i], 32, flags)), i


def test_store_policy_ab_variant_equal():
    """Variant 7 (the earlier non-temporal store policy) writes the same bytes
    as the default; it only exists for A/B timing."""
    frames = np.stack([_rand((1080, 1920, 3), s, "smooth") for s in range(3)])
    want = D.encode(frames, 32, 0, variant=1)
    for v in (0, 5, 7, 11, 12, 13, 14, 15, 16, 17):
        assert np.array_equal(D.encode(frames, 32, 0, variant=v), want), v
    assert np.array_equal(want[1], O.encode_frame(frames[1], 32, 0))


@pytest.mark.parametrize("H,W", [(72, 4104), (64, 72), (61, 77)])
@pytest.mark.parametrize("flags", [0, 1, 2])
def test_decode_zero_skipping(H, W, flags):
    """Index frames whose blocks carry nonzero coefficients only in their first
    Ki rows and Kj columns (random per block, and per 8-block group so whole
    waves share an extent) decode to the same bytes with the zero-skipping
    product kernel, the dense kernel of the A/B library (variant 2) and the
    oracle."""
    rng = np.random.Generator(np.random.PCG64(H * W + flags))
    Hp, Wp = D.padded_shape(H, W)
    nby, nbx = Hp // 8, Wp // 8
    for F in (2,):
        blk = np.full((F, nby, nbx, 8, 8, 3), 128, np.uint8)
        for f in range(F):
            for by in range(nby):
                for g in range(0, nbx, 8):
                    grp = rng.random() < 0.5        # one extent for the whole group of 8 blocks
                    Ki, Kj = rng.integers(1, 9, 2)
                    for bx in range(g, min(g + 8, nbx)):
                        if not grp:
                            Ki, Kj = rng.integers(1, 9, 2)
                        blk[f, by, bx, :Ki, :Kj] = rng.integers(100, 157, (Ki, Kj, 3))
        if flags & 1:   # -x: blocks in place
            k = blk.transpose(0, 1, 3, 2, 4, 5).reshape(F, Hp, Wp, 3)
        else:           # subbands: coefficient (i, j) of block (by, bx) at (i nby + by, j nbx + bx)
            k = blk.transpose(0, 3, 1, 4, 2, 5).reshape(F, Hp, Wp, 3)
        k = np.ascontiguousarray(k)
        got = D.decode(k, H, W, 32, flags)
        assert np.array_equal(got, D.decode(k, H, W, 32, flags, variant=2))
        assert np.array_equal(got[1], O.decode_frame(k[1], H, W, 32, flags))
