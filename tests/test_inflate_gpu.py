"""GPU TIFF strip inflate (vcf_inflate_strips, csrc/vcf_inflate.hip) against
zlib.decompress: every block type (stored, fixed, dynamic), every zlib level and
strategy, strip lengths 0..65536, many strips per launch, and the TIFF files of
the reference's fixtures (the decode side of TIFF.py:33-39)."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inflate(streams, lengths, violations=None):
    from vcf_amd.device import DeviceBuffer, Stream
    from vcf_amd.zlib_gpu import StripInflater
    comp = np.frombuffer(b"".join(streams), np.uint8) if streams else np.zeros(0, np.uint8)
    comp_len = np.array([len(s) for s in streams], np.int32)
    comp_off = np.concatenate([[0], np.cumsum(comp_len)[:-1]]).astype(np.int64)
    out_len = np.array(lengths, np.int32)
    out_off = np.concatenate([[0], np.cumsum(out_len)[:-1]]).astype(np.int64)
    out = DeviceBuffer(max(16, int(out_len.sum())))
    st = Stream()
    StripInflater().inflate_into(comp, comp_off, comp_len, out, out_off, out_len, st, violations=violations)
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


@pytest.mark.parametrize("case", range(5))
def test_rejects_corrupt_code_lengths(case):
    """inflate_table's checks (zlib inftrees.c): over-subscribed and incomplete
    code-length sets, and inflate's missing end-of-block code, each rejected
    with its own status (tests/deflate_corrupt.py; zlib rejects the same
    streams, tests/test_deflate.py::test_zlib_rejects_corrupt_code_lengths)."""
    from deflate_corrupt import CASES
    name, stream, _, status = CASES[case]
    with pytest.raises(ValueError, match=rf"\(status {status}\)"):
        _inflate([stream], [1000])


def test_rejects_bad_strip_tables():
    """A strip table that does not fit its buffers is refused on the host,
    before the kernel runs (no out-of-bounds device reads or writes)."""
    from vcf_amd.device import DeviceBuffer, Stream
    from vcf_amd.zlib_gpu import StripInflater
    b = _data("image", 3000, np.random.default_rng(2))
    c = np.frombuffer(zlib.compress(b, 6), np.uint8)
    out, st, inf = DeviceBuffer(4096), Stream(), StripInflater()
    one = lambda v: np.array([v], np.int64)   # noqa: E731
    for args in ((one(0), one(len(c)), one(0), one(-1)),        # negative output length
                 (one(0), one(-5), one(0), one(3000)),           # negative compressed length
                 (one(10), one(len(c)), one(0), one(3000)),      # strip past the compressed bytes
                 (one(0), one(len(c)), one(2000), one(3000))):   # strip past the output buffer
        with pytest.raises(ValueError):
            inf.inflate_into(c, args[0], args[1], out, args[2], args[3], st)
    inf.inflate_into(c, one(0), one(len(c)), out, one(1000), one(3000), st)   # the same strip, fitting
    got = np.empty(3000, np.uint8)
    out.download(got, offset=1000)
    assert got.tobytes() == b


def test_window_check_reports_no_violations():
    """The window-check build (A/B library, vcf_inflate_strips_wincheck):
    every back-reference and flush read of the 32 KiB output ring lies in its
    valid span -- zero violations -- on streams with matches at every
    distance up to 32 768 (zlib levels 1-9, all strategies, 64 KiB strips,
    long-distance repeats), and the outputs equal the product kernel's."""
    rng = np.random.default_rng(77)
    raw, streams = [], []
    for level in (1, 4, 6, 9):
        for strategy in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_RLE, zlib.Z_FIXED):
            for kind in ("random", "sparse", "text", "image"):
                b = _data(kind, int(rng.integers(30000, 65537)), rng)
                raw.append(b)
                streams.append(_compress(b, level, strategy))
    for d in (1, 2, 257, 4096, 32767, 32768):   # a block repeated at distance d, then again
        blk = rng.integers(0, 256, d if d < 32768 else 32768, dtype=np.uint8).tobytes()
        b = (blk * (65536 // len(blk) + 2))[:65536]
        raw.append(b)
        streams.append(zlib.compress(b, 9))
    viol = np.full(len(streams), 0xFFFFFFFF, np.uint32)
    got = _inflate(streams, [len(b) for b in raw], violations=viol)
    assert got == raw
    assert not viol.any(), np.nonzero(viol)[0]
    assert got == _inflate(streams, [len(b) for b in raw])
