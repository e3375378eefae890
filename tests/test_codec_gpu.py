"""The drop-in CoDec end to end on the GPU: PNG in, the reference's .tif and
_shape.bin bytes out; the reference's .tif in, the reference's decoded
pixels out (tests/golden, made by src/2D-DCT.py itself).  Plus the batched
multi-frame path and the stand-alone deadzone quantizer."""
import os

import numpy as np
import pytest
from PIL import Image

from conftest import golden_cases, load_case
from vcf_amd.codec import parser as P

pytestmark = pytest.mark.gpu


def _args(sub, case_flags=()):
    return P.parse(P.dct_parser(), [sub] + list(case_flags))


def _png(path, rgb):
    Image.fromarray(rgb).save(path)
    return str(path)


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_encode_fn_decode_fn_reproduce_reference_files(tmp_path, case):
    from vcf_amd.codec.dct2d import CoDec
    d = load_case(case)
    src = _png(tmp_path / "original.png", d["rgb"])
    out = str(tmp_path / "encoded")
    n = CoDec(_args("encode", case["flags"])).encode_fn(src, out)
    tif = open(out + ".tif", "rb").read()
    assert tif == bytes(d["tif"]) and n == len(tif) == case["encode_bytes"]
    assert open(out + "_shape.bin", "rb").read() == bytes(d["shape_bin"])
    # decode the reference's own code-stream
    with open(out + ".tif", "wb") as f:
        f.write(bytes(d["tif"]))
    dec = str(tmp_path / "decoded.png")
    m = CoDec(_args("decode", case["flags"])).decode_fn(out, dec)
    assert m == os.path.getsize(dec)
    assert np.array_equal(np.asarray(Image.open(dec).convert("RGB")), d["decoded"])


def test_batched_frames_equal_single_frames(tmp_path):
    from vcf_amd.codec.dct2d import CoDec
    rng = np.random.Generator(np.random.PCG64(7))
    shapes = [(72, 104), (72, 104), (61, 77), (72, 104), (8, 8)]
    pairs = []
    for i, (h, w) in enumerate(shapes):
        pairs.append((_png(tmp_path / f"original_{i:04d}.png", rng.integers(0, 256, (h, w, 3), dtype=np.uint8)),
                      str(tmp_path / f"encoded_{i:04d}")))
    c = CoDec(_args("encode"))
    sizes = c.encode_fns(pairs, batch=3)
    for (src, out), n in zip(pairs, sizes):
        ref = str(tmp_path / "single")
        assert CoDec(_args("encode")).encode_fn(src, ref) == n
        assert open(ref + ".tif", "rb").read() == open(out + ".tif", "rb").read()
    dpairs = [(out, str(tmp_path / f"decoded_{i:04d}.png")) for i, (_, out) in enumerate(pairs)]
    CoDec(_args("decode")).decode_fns(dpairs, batch=2)
    for (out, dec) in dpairs:
        single = str(tmp_path / "single_dec.png")
        CoDec(_args("decode")).decode_fn(out, single)
        assert np.array_equal(np.asarray(Image.open(dec)), np.asarray(Image.open(single)))


def test_non_rgb_input_raises_valueerror(tmp_path):
    from vcf_amd.codec.dct2d import CoDec
    src = str(tmp_path / "gray.png")
    Image.fromarray(np.zeros((16, 16), np.uint8)).save(src)
    with pytest.raises(ValueError):
        CoDec(_args("encode")).encode_fn(src, str(tmp_path / "e"))


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int16, np.int32, np.uint8])
@pytest.mark.parametrize("Q", [1, 7, 32, 64])
def test_deadzone_quantizer_plugin(dtype, Q):
    """A5: (x / Q).astype(int32) with numpy's true-division types; Q * k."""
    from vcf_amd import quant
    rng = np.random.Generator(np.random.PCG64(Q))
    if dtype in (np.float32, np.float64):
        x = (rng.standard_normal(100003) * 900).astype(dtype)
        x[:6] = [0.0, -0.0, Q, -Q, Q - 1e-3, -(Q - 1e-3)]
    else:
        info = np.iinfo(dtype)
        x = rng.integers(max(info.min, -30000), min(info.max, 30000), 100003).astype(dtype)
    k = quant.deadzone_quantize(x, Q)
    assert k.dtype == np.int32 and np.array_equal(k, (x / Q).astype(np.int32))
    k16 = k.astype(np.int16)
    y = quant.deadzone_dequantize(k16, Q)
    assert y.dtype == np.int16 and np.array_equal(y, (Q * k16).astype(np.int16))
    y32 = quant.deadzone_dequantize(k, Q)
    assert y32.dtype == np.int32 and np.array_equal(y32, Q * k)


def test_codec_quantize_surface():
    from vcf_amd.codec.dct2d import CoDec
    c = CoDec(_args("encode", ["-q", "5"]))
    x = np.linspace(-100, 100, 4001, dtype=np.float32).reshape(1, -1, 1)
    k = c.quantize(x)
    assert np.array_equal(k, (x / 5).astype(np.int32))
    assert np.array_equal(c.dequantize(k.astype(np.int16)), (5 * k).astype(np.int16))


def _run(argv):
    import subprocess
    import sys
    from conftest import ROOT
    r = subprocess.run([sys.executable] + argv, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


def test_cli_2d_dct_default_paths():
    """`python 2D-DCT.py encode` / `decode` with the reference's hard-wired
    /tmp/original.png -> /tmp/encoded.tif -> /tmp/decoded.png."""
    from oracle import oracle as O
    from vcf_amd.codec.tiff import imwrite_bytes
    rgb = np.random.Generator(np.random.PCG64(11)).integers(0, 256, (67, 90, 3), dtype=np.uint8)
    Image.fromarray(rgb).save("/tmp/original.png")
    _run(["vcf_amd/cli/2D-DCT.py", "encode", "-q", "16"])
    k = O.encode_frame(rgb, 16, 0)
    assert open("/tmp/encoded.tif", "rb").read() == imwrite_bytes(k)
    _run(["vcf_amd/cli/2D-DCT.py", "decode", "-q", "16"])
    assert np.array_equal(np.asarray(Image.open("/tmp/decoded.png")), O.decode_frame(k, 67, 90, 16, 0))


def test_cli_iii_sequence(tmp_path):
    from oracle import oracle as O
    rng = np.random.Generator(np.random.PCG64(12))
    frames = [rng.integers(0, 256, (40, 56, 3), dtype=np.uint8) for _ in range(5)]
    for i, f in enumerate(frames):
        Image.fromarray(f).save(str(tmp_path / f"original_{i:04d}.png"))
    _run(["vcf_amd/cli/III.py", "encode", "-N", "5", "-o", str(tmp_path / "original_%04d.png")])
    _run(["vcf_amd/cli/III.py", "decode", "-N", "5"])
    for i, f in enumerate(frames):
        k = O.encode_frame(f, 32, 0)
        got = np.asarray(Image.open(f"/tmp/decoded_{i:04d}.png"))
        assert np.array_equal(got, O.decode_frame(k, 40, 56, 32, 0))


@pytest.mark.parametrize("ec,ext", [("CBAAC", ".adpt_arith"), ("CBAHC", ".huf")])
def test_dct_codec_with_context_coders(tmp_path, monkeypatch, ec, ext):
    """2D-DCT -c CBAAC / -c CBAHC (config C2's entropy stage): the indices the
    entropy decoder returns are the encoder's, so decode equals the oracle."""
    from oracle import oracle as O
    from vcf_amd.codec.dct2d import CoDec
    monkeypatch.chdir(tmp_path)
    rgb = np.random.Generator(np.random.PCG64(5)).integers(0, 256, (40, 48, 3), dtype=np.uint8)
    src = _png(tmp_path / "o.png", rgb)
    enc = str(tmp_path / "enc")
    c = CoDec(_args("encode", ["-c", ec]))
    assert c.file_extension == ext
    c.encode_fn(src, enc)
    assert os.path.exists(enc + ext)
    dec = str(tmp_path / "d.png")
    CoDec(_args("decode", ["-c", ec])).decode_fn(enc, dec)
    k = O.encode_frame(rgb, 32, 0)
    assert np.array_equal(np.asarray(Image.open(dec)), O.decode_frame(k, 40, 48, 32, 0))


def test_dct_codec_cbaac_1080p(tmp_path, monkeypatch):
    """Config C2 at its own size: one 1080p frame through -c CBAAC (the reference's
    .adpt_arith, the host coder) -- the code stream decodes to the oracle's indices and
    decode_fn's PNG equals the oracle's reconstruction (the reference-format
    coder was tested at 40 x 48 only under -m gpu)."""
    from oracle import oracle as O
    from vcf_amd.codec.dct2d import CoDec
    from vcf_amd.synthetic import synth_frame
    monkeypatch.chdir(tmp_path)
    H, W = 1080, 1920
    rgb = synth_frame(H, W, seed=7)
    src = _png(tmp_path / "o.png", rgb)
    enc = str(tmp_path / "enc")
    c = CoDec(_args("encode", ["-c", "CBAAC"]))
    c.encode_fn(src, enc)
    d = CoDec(_args("decode", ["-c", "CBAAC"]))
    with open(enc + c.file_extension, "rb") as f:
        got_k = d.decompress(f.read())
    k = O.encode_frame(rgb, 32, 0)
    assert np.array_equal(np.asarray(got_k).reshape(k.shape), k)
    dec = str(tmp_path / "d.png")
    d.decode_fn(enc, dec)
    assert np.array_equal(np.asarray(Image.open(dec)), O.decode_frame(k, H, W, 32, 0))


@pytest.mark.parametrize("n,batch", [(7, 3), (5, 8), (9, 2)])
def test_staged_pipeline_equals_single_frames(tmp_path, n, batch):
    """encode_fns through the pinned double-buffered slots (equal-shaped PNGs)
    writes exactly what encode_fn writes frame by frame."""
    from vcf_amd.codec.dct2d import CoDec
    rng = np.random.default_rng(n * 10 + batch)
    pairs = []
    for i in range(n):
        src = _png(tmp_path / f"in_{i}.png", rng.integers(0, 256, (40, 56, 3), dtype=np.uint8))
        pairs.append((src, str(tmp_path / f"enc_{i}")))
    c = CoDec(_args("encode"))
    sizes = c.encode_fns(pairs, batch=batch, io_threads=4)
    for i, (src, out) in enumerate(pairs):
        ref = str(tmp_path / f"ref_{i}")
        m = CoDec(_args("encode")).encode_fn(src, ref)
        assert sizes[i] == m
        assert open(out + ".tif", "rb").read() == open(ref + ".tif", "rb").read()
        assert open(out + "_shape.bin", "rb").read() == open(ref + "_shape.bin", "rb").read()


def test_staged_pipeline_wide_rows_keep_host_writer(tmp_path):
    """Frames whose rows exceed 64 KB (1-row TIFF strips past 21845 px) are
    beyond the GPU deflate's strips: encode_fns writes them with the host
    writer, and the files still equal encode_fn's."""
    from vcf_amd import zlib_gpu
    from vcf_amd.codec.dct2d import CoDec
    assert not zlib_gpu.covers((8, 21848, 3)) and zlib_gpu.covers((8, 21840, 3))
    rng = np.random.default_rng(5)
    pairs = []
    for i in range(3):
        src = _png(tmp_path / f"in_{i}.png", rng.integers(0, 256, (9, 21850, 3), dtype=np.uint8))
        pairs.append((src, str(tmp_path / f"enc_{i}")))
    sizes = CoDec(_args("encode")).encode_fns(pairs, batch=2, io_threads=2)
    for i, (src, out) in enumerate(pairs):
        ref = str(tmp_path / f"ref_{i}")
        assert sizes[i] == CoDec(_args("encode")).encode_fn(src, ref)
        assert open(out + ".tif", "rb").read() == open(ref + ".tif", "rb").read()


@pytest.mark.parametrize("shape", [(61, 77), (1080, 1920), (9, 21850)])
def test_decode_fns_gpu_inflate_equals_decode_fn(tmp_path, shape):
    """decode_fns inflates -c TIFF strips on the GPU (zlib_gpu.StripInflater,
    straight into the index frames the decode kernel reads): the PNGs equal
    decode_fn's (host inflate) frame for frame, mixed with a file whose TIFF
    the host writes (-x layout of another shape) in the same batch."""
    from vcf_amd.codec.dct2d import CoDec
    rng = np.random.default_rng(shape[0])
    H, W = shape
    pairs, dpairs = [], []
    for i in range(4):
        y = np.arange(H)[:, None, None]
        x = np.arange(W)[None, :, None]
        rgb = np.clip(128 + 60 * np.sin(x / (17.0 + i) + y / 29.0 + np.arange(3)) + rng.normal(0, 9, (H, W, 3)),
                      0, 255).astype(np.uint8)
        src = _png(tmp_path / f"in_{i}.png", rgb)
        out = str(tmp_path / f"enc_{i}")
        CoDec(_args("encode")).encode_fn(src, out)
        pairs.append((out, str(tmp_path / f"dec_{i}.png")))
    extra = _png(tmp_path / "odd.png", rng.integers(0, 256, (33, 35, 3), dtype=np.uint8))
    CoDec(_args("encode")).encode_fn(extra, str(tmp_path / "enc_odd"))
    pairs.append((str(tmp_path / "enc_odd"), str(tmp_path / "dec_odd.png")))
    sizes = CoDec(_args("decode")).decode_fns(pairs, batch=3)
    for i, (enc, dec) in enumerate(pairs):
        ref = str(tmp_path / f"ref_{i}.png")
        CoDec(_args("decode")).decode_fn(enc, ref)
        assert np.array_equal(np.asarray(Image.open(dec)), np.asarray(Image.open(ref))), i
        assert sizes[i] > 0
