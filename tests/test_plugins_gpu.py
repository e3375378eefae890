"""§8(f) row 4 plug-ins on the GPU, through libvcf_amd.so: the drop-in codecs
reproduce the files the reference's own glue wrote (tests/golden/plug_*.npz:
.tif bytes, the LloydMax side files, decoded pixels), the kernels equal the
oracle (oracle/plugins.py, oracle.dct_raw_*) on seeded sweeps, and -t YCrCb
in the transform codecs equals -t YCoCg as in the reference."""
import gzip
import io
import os

import numpy as np
import pytest
from PIL import Image

from oracle import oracle as O
from oracle import plugins as P
from test_plugins import cases, load, params
from vcf_amd.codec import parser as PP

pytestmark = pytest.mark.gpu


def _png(path, rgb):
    Image.fromarray(rgb).save(path)
    return str(path)


def _side():
    with open("/tmp/encoded_params.txt", "rb") as f:
        prm = f.read()
    cents = []
    for c in range(3):
        with gzip.GzipFile(f"/tmp/encoded_centroids_{c}.gz", "r") as f:
            cents.append(np.load(io.BytesIO(f.read()), allow_pickle=False))
    return prm, cents


def _check_side(z):
    prm, cents = _side()
    assert prm == bytes(z["params"])
    for c in range(3):
        assert cents[c].dtype == np.float64 and np.array_equal(cents[c], z[f"centroids_{c}"])


def _codec(module, sub, flags):
    if module == "2D-DCT":
        from vcf_amd.codec.dct2d import CoDec
        return CoDec(PP.parse(PP.dct_parser(quantizer=PP.quantizer_of(flags)), [sub] + flags))
    if module == "LloydMax":
        from vcf_amd.codec.pixel import LloydMaxCoDec
        return LloydMaxCoDec(PP.parse(PP.lloydmax_parser(), [sub] + flags))
    from vcf_amd.codec.pixel import YCrCbCoDec
    return YCrCbCoDec(PP.parse(PP.ycrcb_parser(quantizer=PP.quantizer_of(flags)), [sub] + flags))


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_codecs_reproduce_reference_files(tmp_path, case):
    z = load(case)
    fl = list(case["flags"])
    src = _png(tmp_path / "original.png", z["rgb"])
    out = str(tmp_path / "encoded")
    n = _codec(case["module"], "encode", fl).encode_fn(src, out)
    tif = open(out + ".tif", "rb").read()
    assert tif == bytes(z["tif"]) and n == len(tif)
    if "params" in z.files:
        _check_side(z)
    if "shape_bin" in z.files:
        assert open(out + "_shape.bin", "rb").read() == bytes(z["shape_bin"])
    # decode the reference's own code-stream (side files as the reference left them)
    with open(out + ".tif", "wb") as f:
        f.write(bytes(z["tif"]))
    dec = str(tmp_path / "decoded.png")
    _codec(case["module"], "decode", fl).decode_fn(out, dec)
    assert np.array_equal(np.asarray(Image.open(dec).convert("RGB")), z["decoded"])


@pytest.mark.parametrize("module", ["2D-DCT", "2D-DWT"])
def test_t_ycrcb_equals_ycocg(tmp_path, module):
    rng = np.random.Generator(np.random.PCG64(3))
    rgb = rng.integers(0, 256, (45, 70, 3), dtype=np.uint8)
    src = _png(tmp_path / "in.png", rgb)
    files = {}
    for ct in ("YCoCg", "YCrCb"):
        d = tmp_path / ct
        d.mkdir()
        if module == "2D-DCT":
            from vcf_amd.codec.dct2d import CoDec
            args = lambda sub: PP.parse(PP.dct_parser(), [sub, "-t", ct, "-q", "5"])
        else:
            from vcf_amd.codec.dwt2d import CoDec
            args = lambda sub: PP.parse(PP.dwt_parser(), [sub, "-t", ct, "-l", "2", "-w", "bior4.4"])
        CoDec(args("encode")).encode_fn(src, str(d / "enc"))
        CoDec(args("decode")).decode_fn(str(d / "enc"), str(d / "dec.png"))
        files[ct] = {f: open(d / f, "rb").read() if not f.endswith(".png")
                     else np.asarray(Image.open(d / f)).tobytes() for f in sorted(os.listdir(d))}
    assert files["YCoCg"] == files["YCrCb"]


# ---- kernels vs the oracle -------------------------------------------------
@pytest.mark.parametrize("Q", [1, 2, 5, 32, 255, 256, 70000])
def test_ycrcb_dz_vs_oracle(Q):
    from vcf_amd import plugins as V
    rng = np.random.Generator(np.random.PCG64(Q))
    rgb = rng.integers(0, 256, (67, 131, 3), dtype=np.uint8)
    rgb[0, :8] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 0], [0, 255, 255],
                  [255, 0, 255]]
    k = V.ycrcb_dz_encode(rgb, Q)
    assert np.array_equal(k, P.ycrcb_dz_encode(rgb, Q))
    kk = rng.integers(0, 65536, rgb.shape, dtype=np.uint16)     # arbitrary indices (wrapping)
    assert np.array_equal(V.ycrcb_dz_decode(kk, Q), P.ycrcb_dz_decode(kk, Q))
    assert np.array_equal(V.ycrcb_from_rgb(rgb), P.ycrcb_from_rgb(rgb))
    ycc = rng.integers(0, 256, rgb.shape, dtype=np.uint8)
    assert np.array_equal(V.ycrcb_to_rgb(ycc), P.ycrcb_to_rgb(ycc))


def test_ycrcb_all_colours():
    from vcf_amd import plugins as V
    v = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    assert np.array_equal(V.ycrcb_from_rgb(rgb), P.ycrcb_from_rgb(rgb))
    assert np.array_equal(V.ycrcb_to_rgb(rgb), P.ycrcb_to_rgb(rgb))


RANGES = [(0, 255), (-2048, 2047), (-512, 511), (16, 200), (-3, 3), (-20000, 20000)]


@pytest.mark.parametrize("lo,hi", RANGES)
def test_histogram_kernel_vs_numpy_semantics(lo, hi):
    from vcf_amd import plugins as V
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(hi - lo))
    n = hi - lo + 1
    e = np.linspace(lo, hi, n + 1, dtype=np.float32)
    near = np.concatenate([e, np.nextafter(e, np.float32(-np.inf)), np.nextafter(e, np.float32(np.inf))])
    xs = {np.float32: np.concatenate([near, rng.uniform(lo - 5, hi + 5, 60000)]).astype(np.float32),
          np.int16: rng.integers(max(lo - 3, -32768), min(hi + 4, 32767), 60000).astype(np.int16),
          np.uint16: rng.integers(0, 65535, 60000).astype(np.uint16)}
    if lo >= 0:
        xs[np.uint8] = rng.integers(0, 256, 60000).astype(np.uint8)
    for t, x in xs.items():
        x = x[: (x.size // 3) * 3].reshape(-1, 1, 3)
        d = DeviceBuffer.from_array(x)
        h = V.lm_histogram_device(d, t, x.shape[0], 3, lo, hi)
        d.free()
        for c in range(3):
            assert np.array_equal(h[c], P.histogram(x[:, 0, c], lo, hi)), (t, c)
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "plug_histograms.npz"))
    if (lo, hi) in RANGES[:5]:
        i = RANGES.index((lo, hi))
        x = z[f"f32_x_{i}"]
        d = DeviceBuffer.from_array(x)
        assert np.array_equal(V.lm_histogram_device(d, np.float32, x.size, 1, lo, hi)[0], z[f"f32_h_{i}"])
        d.free()


@pytest.mark.parametrize("dtype,lo,hi,Q", [(np.uint8, 0, 255, 32), (np.uint8, 0, 255, 1), (np.uint8, 16, 200, 5),
                                           (np.int16, 0, 255, 16), (np.int16, -2048, 2047, 3),
                                           (np.float32, 0, 255, 32), (np.float32, -2048, 2047, 16),
                                           (np.float32, -512, 511, 1), (np.uint16, 0, 1000, 7)])
def test_lloydmax_quantize_vs_oracle(dtype, lo, hi, Q):
    from vcf_amd import plugins as V
    rng = np.random.Generator(np.random.PCG64(Q * 7 + hi))
    if dtype == np.float32:
        x = (rng.standard_normal((97, 83, 3)) * (hi - lo) / 6).astype(np.float32)
    elif dtype == np.uint16:
        x = rng.integers(0, 1100, (97, 83, 3)).astype(np.uint16)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(max(info.min, lo - 40), min(info.max, hi + 40) + 1, (97, 83, 3)).astype(dtype)
    k, cents = V.lm_quantize(x, Q, lo, hi)
    ko, co = P.lm_quantize(x, Q, lo, hi)
    assert k.dtype == x.dtype and np.array_equal(k, ko)
    for c in range(3):
        assert np.array_equal(cents[c], co[c])
    ki = np.clip(ko, 0, len(co[0]) - 1).astype(np.int16 if dtype == np.float32 else dtype)
    assert np.array_equal(V.lm_dequantize(ki, cents), P.lm_dequantize(ki, co))


def test_lloydmax_index_out_of_range_raises():
    from vcf_amd import plugins as V
    k = np.zeros((4, 4, 3), np.uint8)
    k[2, 3, 1] = 8
    with pytest.raises(IndexError):
        V.lm_dequantize(k, [np.arange(8.0)] * 3)
    k16 = np.full((4, 4, 3), -1, np.int16)      # numpy's negative indices count from the end
    assert np.array_equal(V.lm_dequantize(k16, [np.arange(8.0) + 0.5] * 3), np.full((4, 4, 3), 7, np.int16))


@pytest.mark.parametrize("B,flags", [(8, 0), (8, 1), (8, 2), (16, 3), (7, 0), (12, 2), (13, 1)])
def test_raw_dct_vs_oracle(B, flags):
    from vcf_amd import dct as D
    from vcf_amd.device import DeviceBuffer
    rng = np.random.Generator(np.random.PCG64(B * 4 + flags))
    rgb = rng.integers(0, 256, (53, 91, 3), dtype=np.uint8)
    H, W = rgb.shape[:2]
    Hp, Wp = D.padded_shape(H, W, B)
    d = DeviceBuffer.from_array(rgb)
    coef = D.raw_encode_device(d, 1, H, W, flags, block_size=B)
    got = coef.download(np.empty((Hp, Wp, 3), np.float32))
    assert np.array_equal(got.view(np.uint32), O.dct_raw_encode_b(rgb, B, flags).view(np.uint32))
    y = (rng.standard_normal((Hp, Wp, 3)) * 300).astype(np.int16)
    dy = DeviceBuffer.from_array(y)
    rec = D.raw_decode_device(dy, 1, H, W, flags, block_size=B)
    assert np.array_equal(rec.download(np.empty((H, W, 3), np.uint8)), O.dct_raw_decode_b(y, H, W, B, flags))
    for b in (d, coef, dy, rec):
        b.free()


def test_dct_lloydmax_1080p_round_trip_vs_oracle(tmp_path):
    """A 1080p frame through the -a LloydMax codec: indices and reconstruction equal the oracle."""
    from vcf_amd.codec.dct2d import CoDec
    rng = np.random.Generator(np.random.PCG64(11))
    y, x = np.mgrid[0:1080, 0:1920].astype(np.float64)
    rgb = np.clip(np.stack([128 + 60 * np.sin(x / 97 + c) + 50 * np.cos(y / 61 - c) for c in range(3)], -1)
                  + rng.normal(0, 4, (1080, 1920, 3)), 0, 255).astype(np.uint8)
    fl = ["-a", "LloydMax", "-m", "-2048", "-n", "2047", "-q", "16"]
    c = _codec("2D-DCT", "encode", fl)
    k = c.encode_lm(rgb)
    coef = O.dct_raw_encode_b(rgb, 8, 0)
    ko, co = P.lm_quantize(coef, 16, -2048, 2047)
    assert np.array_equal(k, ko.astype(np.uint8))
    rec = _codec("2D-DCT", "decode", fl).decode_lm(k, rgb.shape)
    yo = P.lm_dequantize(k.astype(np.int16), co)
    assert np.array_equal(rec, O.dct_raw_decode_b(yo, 1080, 1920, 8, 0))
