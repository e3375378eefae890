"""GPU TIFF strip inflate (vcf_inflate_strips, csrc/vcf_inflate.hip) against
zlib.decompress: every block type (stored, fixed, dynamic), every zlib level and
strategy, strip lengths 0..65536, many strips per launch, and the TIFF files of
the reference's fixtures (the decode side of TIFF.py:33-39)."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inflate(streams, lengths):
    from vcf_amd.device import DeviceBuffer, Stream
    from vcf_amd.zlib_gpu import StripInflater
    comp = np.frombuffer(b"".join(streams), np.uint8) if streams else np.zeros(0, np.uint8)
    comp_len = np.array([len(s) for s in streams], np.int32)
    comp_off = np.concatenate([[0], np.cumsum(comp_len)[:-1]]).astype(np.int64)
    out_len = np.array(lengths, np.int32)
    out_off = np.concatenate([[0], np.cumsum(out_len)[:-1]]).astype(np.int64)
    out = DeviceBuffer(max(16, int(out_len.sum())))
    st = Stream()
    StripInflater().inflate_into(comp, comp_off, comp_len, out, out_off, out_len, st)
    host = np.empty(int(out_len.sum()), np.uint8)
    if host.size:
        out.download(host)
    return [host[o:o + n].tobytes() for o, n in zip(out_off, out_len)]


def _data(kind, n, rng):
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "sparse":
        a = np.full(n, 128, np.uint8)
        m = rng.random(n) < 0.03
        a[m] = rng.integers(100, 160, int(m.sum()))
        return a.tobytes()
    if kind == "text":
        return (b"the quick brown fox jumps over the lazy dog " * (n // 44 + 1))[:n]
    x = np.arange(n)
    return np.clip(128 + 60 * np.sin(x / 37.0) + rng.normal(0, 4, n), 0, 255).astype(np.uint8).tobytes()


def _compress(b, level, strategy):
    c = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    return c.compress(b) + c.flush()


@pytest.mark.parametrize("strategy", [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE,
                                      zlib.Z_FILTERED])
def test_levels_and_strategies(strategy):
    rng = np.random.default_rng(strategy + 1)
    raw, streams = [], []
    for level in range(0, 10):
        for kind in ("random", "sparse", "text", "image"):
            b = _data(kind, int(rng.integers(1, 70000)), rng)
            raw.append(b)
            streams.append(_compress(b, level, strategy))
    got = _inflate(streams, [len(b) for b in raw])
    for i, (g, w) in enumerate(zip(got, raw)):
        assert g == w, i


@pytest.mark.parametrize("n", [0, 1, 2, 3, 257, 258, 1023, 1024, 1025, 32767, 32768, 32769, 65535, 65536])
def test_lengths(n):
    rng = np.random.default_rng(n)
    raw = [_data(k, n, rng) for k in ("random", "sparse", "image")]
    got = _inflate([zlib.compress(b, 6) for b in raw], [n] * 3)
    assert got == raw


def test_many_strips_and_unaligned_offsets():
    rng = np.random.default_rng(9)
    raw = [_data(("sparse", "image", "random")[i % 3], int(rng.integers(1, 9000)), rng) for i in range(700)]
    assert _inflate([zlib.compress(b, 6) for b in raw], [len(b) for b in raw]) == raw


def test_rejects_what_zlib_rejects():
    b = _data("image", 5000, np.random.default_rng(1))
    c = bytearray(zlib.compress(b, 6))
    bad_adler = bytes(c[:-1] + bytes([c[-1] ^ 1]))
    for streams, n in (([bad_adler], 5000), ([bytes(c)], 4999), ([bytes(c)], 5001), ([b"\x00\x00" + bytes(c[2:])], 5000)):
        with pytest.raises(ValueError):
            _inflate(streams, [n])


def test_reference_tiff_strips():
    """The strips of the reference's own .tif files (tests/golden/dct_*.npz 'tif'):
    inflated on the GPU they give the fixture's index array."""
    import glob
    import os
    from conftest import GOLDEN
    from vcf_amd.codec.tiff import tiff_strips
    streams, want = [], []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "dct_*.npz")))[:20]:
        z = np.load(f, allow_pickle=False)
        info = tiff_strips(z["tif"].tobytes())
        if info is None:
            continue
        shape, dtype, offs, counts, strip_bytes = info
        k = np.ascontiguousarray(z["k"]).reshape(-1).view(np.uint8).tobytes()
        for j, (o, c) in enumerate(zip(offs, counts)):
            streams.append(z["tif"].tobytes()[o:o + c])
            want.append(k[j * strip_bytes:(j + 1) * strip_bytes])
    got = _inflate(streams, [len(w) for w in want])
    assert got == want and len(got) > 20
