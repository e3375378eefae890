"""Single-frame row-stripe sharding with the HIP kernels (SURVEY.md §8(e),
vcf_amd/codec/stripes.py): stripes coded by the real kernels equal the
whole-frame kernels and the oracle; two ranks share this box's GPU over the
host group (RCCL needs one device per rank: the 8-GPU path is the driver's)."""
import numpy as np
import pytest

from oracle import oracle as O
from vcf_amd import dct as D
from vcf_amd.codec import stripes as S
from vcf_amd.dct import VCF_DCT_NO_SUBBANDS, VCF_DCT_PERCEPTUAL

pytestmark = pytest.mark.gpu


def _img(H, W, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, (H, W, 3), dtype=np.uint8)


@pytest.mark.parametrize("H,W,B,P", [(2160, 3840, 8, 8), (1083, 1917, 8, 3), (517, 300, 16, 4), (45, 70, 8, 8)])
@pytest.mark.parametrize("flags", [0, VCF_DCT_NO_SUBBANDS | VCF_DCT_PERCEPTUAL])
def test_stripes_equal_whole_frame_gpu(H, W, B, P, flags):
    from vcf_amd.device import set_device
    set_device(0)
    rgb = _img(H, W, H + W + P)
    Hp, Wp = D.padded_shape(H, W, B)
    whole = D.encode(rgb, 32, flags, block_size=B)
    k = np.zeros((Hp, Wp, 3), np.uint8)
    parts = []
    for r in range(P):
        by0, by1 = S.block_rows(H, B, r, P)
        if by1 == by0:
            continue
        ks = D.encode(S.stripe_pixels(rgb, by0, by1, B), 32, flags, block_size=B)
        S.place_stripe(k, ks, by0, by1, B, flags)
        parts.append(D.decode(S.take_stripe(whole, by0, by1, B, flags), B * (by1 - by0), W, 32, flags,
                              block_size=B))
    assert np.array_equal(k, whole)
    top = (Hp - H) // 2
    y = np.concatenate(parts)[top:top + H]
    assert np.array_equal(y, D.decode(whole, H, W, 32, flags, block_size=B))
    if H * W <= 600_000:
        assert np.array_equal(whole, O.encode_frame_b(rgb, B, 32, flags))
        assert np.array_equal(y, O.decode_frame_b(whole, H, W, B, 32, flags))


def _worker(rank, world, rgb, kk, Q, flags):
    from vcf_amd.codec import shard
    from vcf_amd.device import set_device
    set_device(0)                           # both ranks share this box's one GPU
    g = shard.Group("host")
    k = S.encode_frame(rgb, g, Q, flags)
    y = S.decode_frame(kk, rgb.shape[0], rgb.shape[1], g, Q, flags)
    g.close()
    return k, y


def test_stripes_two_ranks_real_kernels():
    from _dist import run_ranks
    H, W = 301, 522
    rgb = _img(H, W, 17)
    kk = O.encode_frame_b(rgb, 8, 24, 0)
    res = run_ranks(_worker, 2, rgb, kk, 24, 0)
    k, y = res[0]
    assert res[1] == (None, None)
    assert np.array_equal(k, kk)
    assert np.array_equal(y, O.decode_frame_b(kk, H, W, 8, 24, 0))
