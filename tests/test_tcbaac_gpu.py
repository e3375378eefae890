"""Tiled CBAAC on the GPU (vcf_amd/csrc/vcf_cbaac_gpu.hip through the C ABI).

- The model, segment by segment, equals the reference's own AdaptiveModel /
  ContextManager run on each segment from scratch (traces made by executing
  the reference's classes: tests/golden/make_golden_cbaac.py tiled).
- Every segment's bytes equal the host serial coder's (vcf_cbaac_encode) on
  that segment alone; the GPU decoder inverts both exactly.
- Edge cases: empty, 1 symbol, partial last chunk / segment, runs, uniform
  noise (no compression), orders 0 and 1, long segments with rescales.
- The DCT CoDec with `-c TCBAAC`: the indices never leave HBM; the decoded
  frame equals the oracle's.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from vcf_amd import tcbaac as T

pytestmark = pytest.mark.gpu

_MAN = json.load(open(os.path.join(GOLDEN, "manifest_cbaac_tiled.json")))


@pytest.mark.parametrize("case", _MAN["cases"], ids=lambda c: f"{c['stream']}_o{c['order']}")
def test_segment_traces_equal_reference_classes(case):
    d = np.load(os.path.join(GOLDEN, "cbaac_tiled.npz"))
    sym = d[f"sym_{case['stream']}"]
    ref = d[f"trace_{case['stream']}_o{case['order']}"]
    got = T.TiledCoder(case["order"], case["seg_len"]).trace(sym)
    bad = np.nonzero(np.any(got != ref, axis=1))[0]
    assert bad.size == 0, (bad[:5], got[bad[:3]], ref[bad[:3]])


def _streams():
    rng = np.random.Generator(np.random.PCG64(5))
    lap = np.clip(np.rint(rng.laplace(128, 2.5, 300_001)), 0, 255).astype(np.uint8)
    skew = np.where(rng.random(70_000) < 0.985, 128, rng.integers(0, 256, 70_000)).astype(np.uint8)
    return {
        "laplace": lap,
        "skewed": skew,
        "uniform": rng.integers(0, 256, 40_000, dtype=np.uint8),
        "runs": np.repeat(rng.integers(0, 256, 300, dtype=np.uint8), 97),
        "const255": np.full(5000, 255, np.uint8),
        "one": np.array([17], np.uint8),
        "tiny": rng.integers(0, 256, 255, dtype=np.uint8),
        "empty": np.zeros(0, np.uint8),
    }


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("seg_len", [256, 4096, 1 << 17])
def test_segments_equal_host_coder_and_round_trip(order, seg_len):
    coder = T.TiledCoder(order, seg_len)
    for name, sym in _streams().items():
        if seg_len == 256 and sym.size > 50_000:
            sym = sym[:50_000 + 77]
        sizes, payload = coder.encode(sym)
        host = T.host_segments(sym, order, seg_len)
        assert list(sizes) == [len(h) for h in host], name
        assert payload == b"".join(host), name
        assert np.array_equal(coder.decode(payload, sizes, sym.size), sym), name


def test_decode_with_one_fresh_coder_per_call():
    sym = _streams()["laplace"]
    sizes, payload = T.TiledCoder(0, 8192).encode(sym)
    assert np.array_equal(T.TiledCoder(0, 8192).decode(payload, sizes, sym.size), sym)


def test_codec_container_and_errors():
    rng = np.random.Generator(np.random.PCG64(2))
    img = np.clip(np.rint(rng.laplace(128, 3, (96, 130, 3))), 0, 255).astype(np.uint8)
    c = T.TiledCBAACCodec(order=1, seg_len=4096)
    b = c.compress(img)
    assert c.file_extension == ".tadpt_arith"
    assert np.array_equal(c.decompress(b.getvalue()), img)
    assert np.array_equal(T.TiledCBAACCodec().decompress(b.getvalue()), img)   # order/seg_len from the header
    with pytest.raises(NotImplementedError):
        T.TiledCoder(2, 4096).encode(img.ravel())
    with pytest.raises(ValueError):
        T.TiledCoder(0, 1000).encode(img.ravel())                              # not a multiple of 256


def test_dct_codec_with_tcbaac_frame(tmp_path):
    from PIL import Image

    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    rgb = synth_frame(1080, 1920, 3)
    src = str(tmp_path / "f.png")
    Image.fromarray(rgb).save(src)
    enc = CoDec(P.parse(P.dct_parser(), ["encode", "-c", "TCBAAC"]))
    nbytes = enc.encode_fn(src, str(tmp_path / "enc"))
    data = open(str(tmp_path / "enc.tadpt_arith"), "rb").read()
    assert nbytes == len(data)
    k = O.encode_frame(rgb, 32, 0)
    shape, order, seg_len, sizes, payload = T.unpack(data)
    assert shape == k.shape and order == 0 and seg_len == T.DEFAULT_SEG
    assert payload == b"".join(T.host_segments(k, 0, seg_len))
    dec = CoDec(P.parse(P.dct_parser(), ["decode", "-c", "TCBAAC"]))
    dec.decode_fn(str(tmp_path / "enc"), str(tmp_path / "out.png"))
    out = np.asarray(Image.open(str(tmp_path / "out.png")))
    assert np.array_equal(out, O.decode_frame(k, 1080, 1920, 32, 0))


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("seg_len", [256, 4096, 32768])
def test_prior_segments_equal_host_coder_and_round_trip(order, seg_len):
    """Container version 2: the GPU prior equals the host formula; every
    segment's bytes equal vcf_cbaac_encode_prior of that segment; the GPU
    decoder inverts them."""
    coder = T.TiledCoder(order, seg_len, prior=True)
    for name, sym in _streams().items():
        if seg_len == 256 and sym.size > 50_000:
            sym = sym[:50_000 + 77]
        sizes, payload = coder.encode(sym)
        prior = T.prior_of(sym)
        assert np.array_equal(coder.last_prior, prior), name
        host = T.host_segments_prior(sym, prior, seg_len, order)
        assert list(sizes) == [len(h) for h in host], name
        assert payload == b"".join(host), name
        assert np.array_equal(coder.decode(payload, sizes, sym.size, prior), sym), name


def test_prior_codec_on_dct_indices():
    """A 1080p frame's indices through the version-2 codec: round trip, and
    short segments cost less rate than with fresh models."""
    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    k = O.encode_frame(synth_frame(1080, 1920, 3), 32, 0)
    c = T.TiledCBAACCodec(order=0, seg_len=8192, prior=True)
    data = c.compress(k).getvalue()
    assert np.array_equal(T.TiledCBAACCodec().decompress(data), k)
    fresh = T.TiledCBAACCodec(order=0, seg_len=8192).compress(k).getvalue()
    assert len(data) < 0.7 * len(fresh)
    with pytest.raises(NotImplementedError):
        T.TiledCoder(2, 4096, prior=True)


def test_dct_codec_with_tcbaacp_frame(tmp_path):
    """-c TCBAACP: the DCT indices coded on the GPU with models seeded by the
    frame's prior rows (version 3); the file's segments equal the host
    coder's, decoding gives the oracle frame."""
    from PIL import Image

    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    rgb = synth_frame(1080, 1920, 4)
    src = str(tmp_path / "f.png")
    Image.fromarray(rgb).save(src)
    CoDec(P.parse(P.dct_parser(), ["encode", "-c", "TCBAACP"])).encode_fn(src, str(tmp_path / "enc"))
    data = open(str(tmp_path / "enc.tadpt_arith"), "rb").read()
    k = O.encode_frame(rgb, 32, 0)
    shape, order, seg_len, sizes, payload, prior = T._parse(data)
    assert shape == k.shape and order == 0 and seg_len == T.CLASS_SEG
    assert np.array_equal(prior, T.prior_of(k, T.PRIOR_CLASSES, seg_len))   # container version 3
    assert payload == b"".join(T.host_segments_prior(k, prior, seg_len))
    CoDec(P.parse(P.dct_parser(), ["decode", "-c", "TCBAACP"])).decode_fn(str(tmp_path / "enc"),
                                                                         str(tmp_path / "out.png"))
    out = np.asarray(Image.open(str(tmp_path / "out.png")))
    assert np.array_equal(out, O.decode_frame(k, 1080, 1920, 32, 0))


@pytest.mark.parametrize("prior", [False, True])
def test_frames_on_several_streams_equal_one_by_one(prior):
    """encode_frames_device: frames coded concurrently on library streams give
    each frame's stream exactly as coding it alone."""
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(9))
    n, F = 70_000, 5
    frames = [np.where(rng.random(n) < 0.95 - 0.1 * f, 128, rng.integers(0, 256, n)).astype(np.uint8)
              for f in range(F)]
    buf = DeviceBuffer.from_array(np.concatenate(frames))
    got = T.encode_frames_device(buf, F, n, 0, 8192, prior=prior, streams=3)
    for f in range(F):
        c = T.TiledCoder(0, 8192, prior=prior)
        sizes, payload = c.encode(frames[f])
        assert list(got[f][0]) == list(sizes) and got[f][1] == payload, f
        if prior:
            assert np.array_equal(got[f][2], T.prior_of(frames[f]))
            assert np.array_equal(c.decode(payload, sizes, n, got[f][2]), frames[f])


@pytest.mark.parametrize("prior", [False, True])
def test_frames_with_unaligned_starts(prior):
    """Frames of 61x77x3 symbols (n % 4 = 1) back to back: every frame after
    the first starts at an address that is not a multiple of 4, and every
    frame's stream must still equal coding it alone (and so the host coder's).
    Decoding into an unaligned destination must give the symbols back too."""
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(11))
    n, F = 61 * 77 * 3, 3
    assert n % 4
    frames = [np.clip(np.rint(rng.laplace(128, 1.5 + f, n)), 0, 255).astype(np.uint8) for f in range(F)]
    buf = DeviceBuffer.from_array(np.concatenate([np.zeros(1, np.uint8)] + frames))   # frame 0 unaligned too
    got = T.encode_frames_device(buf, F, n, 0, 256, prior=prior, streams=2, offset=1)
    for f in range(F):
        want = (T.host_segments_prior(frames[f], T.prior_of(frames[f]), 256) if prior
                else T.host_segments(frames[f], 0, 256))
        assert list(got[f][0]) == [len(h) for h in want], f
        assert got[f][1] == b"".join(want), f
    c = T.TiledCoder(0, 256, prior=prior)
    dec = DeviceBuffer(n + 3)
    for f in range(F):
        with c.lock:
            c.decode_to_device(got[f][1], got[f][0], n, _Shifted(dec, 3), got[f][2])
            out = np.empty(n, np.uint8)
            dec.download(out, c.stream, offset=3)
            c.stream.synchronize()
        assert np.array_equal(out, frames[f]), f


class _Shifted:
    """A view of a DeviceBuffer `off` bytes in (an unaligned destination)."""

    def __init__(self, buf, off):
        self.buf, self.off = buf, off

    @property
    def ptr(self):
        return self.buf.address(self.off)


@pytest.mark.parametrize("codec", ["TCBAAC", "TCBAACP"])
def test_threaded_encode_fns_decode_fns(tmp_path, codec):
    """The DCT CoDec drives the entropy codec from a thread pool
    (encode_fns/decode_fns): with one shared tiled coder the frames must not
    mix (the coder's scratch and stream are shared, now locked)."""
    from PIL import Image

    from oracle import oracle as O
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    rng = np.random.Generator(np.random.PCG64(12))
    H, W, n = 64, 88, 12
    frames = []
    for i in range(n):
        f = np.clip(np.rint(rng.normal(128 + 5 * i, 20 + i, (H, W, 3))), 0, 255).astype(np.uint8)
        frames.append(f)
        Image.fromarray(f).save(str(tmp_path / f"in_{i}.png"))
    pairs = [(str(tmp_path / f"in_{i}.png"), str(tmp_path / f"enc_{i}")) for i in range(n)]
    enc = CoDec(P.parse(P.dct_parser(), ["encode", "-c", codec]))
    enc.encode_fns(pairs, batch=5, io_threads=8)
    for i in range(n):
        k = O.encode_frame(frames[i], 32, 0)
        data = open(str(tmp_path / f"enc_{i}.tadpt_arith"), "rb").read()
        assert np.array_equal(T.TiledCBAACCodec().decompress(data), k), i
    dpairs = [(str(tmp_path / f"enc_{i}"), str(tmp_path / f"dec_{i}.png")) for i in range(n)]
    dec = CoDec(P.parse(P.dct_parser(), ["decode", "-c", codec]))
    dec.decode_fns(dpairs, batch=5, io_threads=8)
    for i in range(n):
        got = np.asarray(Image.open(str(tmp_path / f"dec_{i}.png")))
        assert np.array_equal(got, O.decode_frame(O.encode_frame(frames[i], 32, 0), H, W, 32, 0)), i


@pytest.mark.parametrize("prior", [False, True])
@pytest.mark.parametrize("seg_len", [256, 4096, 32768])
def test_lane_kernels_equal_wave_kernels(prior, seg_len):
    """Order 0 codes one segment per lane (vcf_cbaac_tiled_set_variant(2); the
    default from 2048 segments on) or one per wave (1): identical streams, and
    each decoder inverts the other's output; long segments cross several
    model rescales."""
    from vcf_amd import _lib as L
    rng = np.random.Generator(np.random.PCG64(seg_len + prior))
    n = 200_003
    base = np.where(rng.random(n) < 0.97, 128, rng.integers(0, 256, n))
    sym = np.clip(base + (rng.random(n) < 0.3) * rng.integers(-2, 3, n), 0, 255).astype(np.uint8)
    sym[:5000] = rng.integers(0, 256, 5000)           # a noisy stretch: wide ranges, frequent rescales
    sym[-70:] = 255
    try:
        L.call("vcf_cbaac_tiled_set_variant", 1)
        c1 = T.TiledCoder(0, seg_len, prior=prior)
        s1, p1 = c1.encode(sym)
        L.call("vcf_cbaac_tiled_set_variant", 2)
        c0 = T.TiledCoder(0, seg_len, prior=prior)
        s0, p0 = c0.encode(sym)
        assert list(s0) == list(s1) and p0 == p1
        pr = c0.last_prior if prior else None
        assert np.array_equal(c0.decode(p0, s0, n, pr), sym)     # lane decoder
        L.call("vcf_cbaac_tiled_set_variant", 1)
        assert np.array_equal(c1.decode(p0, s0, n, pr), sym)     # wave decoder, same stream
    finally:
        L.call("vcf_cbaac_tiled_set_variant", 0)


def test_lane_kernels_on_dct_indices_many_segments():
    """A 1080p frame's indices in 256-symbol segments (24 300 segments: the
    automatic choice codes one per lane, 380 waves): every segment equals the
    host coder seeded with the frame's prior."""
    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    k = O.encode_frame(synth_frame(1080, 1920, 5), 32, 0).ravel()
    c = T.TiledCoder(0, 256, prior=True)
    sizes, payload = c.encode(k)
    host = T.host_segments_prior(k, T.prior_of(k), 256)
    assert list(sizes) == [len(h) for h in host]
    assert payload == b"".join(host)
    assert np.array_equal(c.decode(payload, sizes, k.size, c.last_prior), k)


@pytest.mark.parametrize("variant", [1, 2])
def test_batch_decode_frames(variant):
    """vcf_cbaac_tiled_decode_frames: a batch of prior-seeded frames decoded in
    one launch (segment offsets into one payload buffer, outputs at a stride)
    gives every frame back, with either kernel."""
    from vcf_amd import _lib as L
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(21))
    n, F, seg = 10_001, 6, 1024
    frames = [np.clip(np.rint(rng.laplace(128, 0.7 + f, n)), 0, 255).astype(np.uint8) for f in range(F)]
    enc = T.encode_frames_device(DeviceBuffer.from_array(np.concatenate(frames)), F, n, 0, seg, prior=True)
    ns = T.n_segments(n, seg)
    payload = b"".join(e[1] for e in enc)
    offs, base = [], 0
    for e in enc:
        o = np.concatenate([[0], np.cumsum(e[0])]) + base
        offs.append(o)
        base += len(e[1])
    offs = np.concatenate(offs).astype(np.int64)
    assert offs.size == F * (ns + 1)
    priors = np.stack([e[2] for e in enc]).astype(np.uint16)
    src, doffs, dpr = (DeviceBuffer.from_array(np.frombuffer(payload, np.uint8)), DeviceBuffer.from_array(offs),
                       DeviceBuffer.from_array(priors))
    stride = n + 3                                   # unaligned output frames
    out = DeviceBuffer(F * stride)
    try:
        L.call("vcf_cbaac_tiled_set_variant", variant)
        L.call("vcf_cbaac_tiled_decode_frames", src.ptr, doffs.ptr, F, n, 0, dpr.ptr, seg, out.ptr, stride, None)
        got = out.download(np.empty(F * stride, np.uint8))
    finally:
        L.call("vcf_cbaac_tiled_set_variant", 0)
    for f in range(F):
        assert np.array_equal(got[f * stride:f * stride + n], frames[f]), f


# ---- version 3: prior classes ---------------------------------------------------------

def _dct_indices(H=1080, W=1920, seed=5):
    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    return O.encode_frame(synth_frame(H, W, seed), 32, 0).ravel()


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("order,seg_len,nclass", [(0, 4096, 8), (0, 256, 3), (1, 4096, 8), (0, 8192, 200)])
def test_class_prior_segments_equal_host_coder(variant, order, seg_len, nclass):
    """Container version 3: the GPU's prior rows equal the host formula over
    each class's segments; every segment's bytes equal
    vcf_cbaac_encode_prior of that segment with its class's row, with one
    wave (1) or one lane (2, order 0) per segment; both decoders invert it.
    nclass = 200 > some frames' segment count leaves rows with no segments."""
    from vcf_amd import _lib as L
    rng = np.random.Generator(np.random.PCG64(seg_len + nclass))
    lap = np.clip(np.rint(rng.laplace(128, 1.5, 300_001)), 0, 255).astype(np.uint8)
    lap[100_000:140_000] = 128
    for name, sym in (("dct", _dct_indices()), ("laplace", lap)):
        try:
            L.call("vcf_cbaac_tiled_set_variant", variant)
            c = T.TiledCoder(order, seg_len, prior=True, nclass=nclass)
            sizes, payload = c.encode(sym)
            prior = T.prior_of(sym, nclass, seg_len)
            assert np.array_equal(c.last_prior, prior), name
            host = T.host_segments_prior(sym, prior, seg_len, order)
            assert list(sizes) == [len(h) for h in host], name
            assert payload == b"".join(host), name
            assert np.array_equal(c.decode(payload, sizes, sym.size, prior), sym), name
        finally:
            L.call("vcf_cbaac_tiled_set_variant", 0)


def test_class_priors_cut_the_rate_of_short_segments():
    """On a 1080p frame's DCT indices (subband layout) 4096-symbol segments
    with 8 prior rows cost at most 3 % over the serial stream (one prior row:
    about +12 %), container bytes included."""
    from vcf_amd.cbaac import encode_symbols
    k = _dct_indices()
    serial = len(encode_symbols(k, 0))
    c8 = T.TiledCBAACCodec(0, T.CLASS_SEG, prior=True, nclass=T.PRIOR_CLASSES)
    c1 = T.TiledCBAACCodec(0, T.CLASS_SEG, prior=True)
    b8 = len(c8.compress(k.reshape(1080, 1920, 3)).getvalue())
    b1 = len(c1.compress(k.reshape(1080, 1920, 3)).getvalue())
    assert b8 <= 1.03 * serial, (b8, serial)
    assert b1 > b8


def test_frame_batch_with_classes_equals_one_by_one():
    """FrameBatch / encode_frames_device with prior classes (one launch per
    stage for the batch, unaligned frame starts) equals coding each frame
    alone; the batched decode (vcf_cbaac_tiled_decode_classes) inverts it."""
    from vcf_amd import _lib as L
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(33))
    n, F, seg, K = 61 * 77 * 3, 5, 1024, 4
    frames = [np.clip(np.rint(rng.laplace(128, 0.5 + f, n)), 0, 255).astype(np.uint8) for f in range(F)]
    buf = DeviceBuffer.from_array(np.concatenate([np.zeros(1, np.uint8)] + frames))
    got = T.encode_frames_device(buf, F, n, 0, seg, prior=True, offset=1, nclass=K)
    for f in range(F):
        c = T.TiledCoder(0, seg, prior=True, nclass=K)
        s, p = c.encode(frames[f])
        assert list(got[f][0]) == list(s) and got[f][1] == p, f
        assert np.array_equal(got[f][2], c.last_prior), f
    ns = T.n_segments(n, seg)
    payload = b"".join(e[1] for e in got)
    offs, base = [], 0
    for e in got:
        offs.append(np.concatenate([[0], np.cumsum(e[0])]) + base)
        base += len(e[1])
    offs = np.concatenate(offs).astype(np.int64)
    priors = np.stack([e[2] for e in got]).astype(np.uint16)
    assert priors.shape == (F, K, 256)
    src, doffs, dpr = (DeviceBuffer.from_array(np.frombuffer(payload, np.uint8)), DeviceBuffer.from_array(offs),
                       DeviceBuffer.from_array(priors))
    out = DeviceBuffer(F * n)
    L.call("vcf_cbaac_tiled_decode_classes", src.ptr, doffs.ptr, F, n, 0, dpr.ptr, K, seg, out.ptr, n, None)
    dec = out.download(np.empty(F * n, np.uint8))
    assert offs.size == F * (ns + 1)
    for f in range(F):
        assert np.array_equal(dec[f * n:(f + 1) * n], frames[f]), f


def test_tcbaacp_codec_is_version_3(tmp_path):
    """-c TCBAACP writes container version 3 (8 prior rows, 4096-symbol
    segments) and decodes it; version-2 streams still decode."""
    import struct
    k = _dct_indices(272, 480, 2).reshape(272, 480, 3)
    from vcf_amd.codec.dct2d import _tcbaac_prior
    codec = _tcbaac_prior()
    data = codec.compress(k).getvalue()
    shape, order, seg_len, sizes, payload, prior = T._parse(data)
    assert struct.unpack_from("<I", data, 4 + 4 * 3 + 4)[0] == T.VERSION_CLASSES
    assert seg_len == T.CLASS_SEG and prior.shape == (T.PRIOR_CLASSES, 256)
    assert np.array_equal(codec.decompress(data), k)
    v2 = T.TiledCBAACCodec(0, 8192, prior=True).compress(k).getvalue()
    assert np.array_equal(codec.decompress(v2), k)


def test_frame_batch_headers_equal_pack():
    """FrameBatch.headers (the whole batch's version-3 headers from two native
    calls) equals pack() of every frame, and header + payload decodes."""
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(8))
    shape, F = (16, 40, 3), 6
    n = int(np.prod(shape))
    frames = np.clip(np.rint(rng.laplace(128, 2.0, (F, n))), 0, 255).astype(np.uint8)
    fb = T.FrameBatch(F, n, 0, 256, prior=True, nclass=3)
    fb.launch(DeviceBuffer.from_array(frames))
    heads = fb.headers(shape)
    got = fb.download()
    for f in range(F):
        assert heads[f] == fb.header(f, shape) == T.pack(shape, 0, 256, got[f][0], b"", got[f][2]), f
        assert np.array_equal(T.TiledCBAACCodec(0, 256).decompress(heads[f] + got[f][1]), frames[f].reshape(shape))
