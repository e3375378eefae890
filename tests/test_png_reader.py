"""The library's PNG reader (vcf_amd/csrc/vcf_png.cpp, host code, no GPU)
against PIL's convert("RGB") -- the array EIC.encode_read_fn hands on
(entropy_image_coding.py:51-65, assumption A9): every colour type PIL writes
at 8 bits, all five scanline filters (a small test-only writer forces each),
odd sizes, multi-IDAT files; corrupt files raise; PNGs outside the covered
set (16-bit) fall back to PIL through eic.read_image."""
import io
import os
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

from conftest import ROOT
from vcf_amd.codec import eic


def _pil_rgb(png: bytes):
    return np.asarray(Image.open(io.BytesIO(png)).convert("RGB"))


def _native(png: bytes, tmp_path, name="x.png"):
    p = tmp_path / name
    p.write_bytes(png)
    img, n = eic._read_png_native(str(p))
    assert n == len(png)
    return img


def _pil_png(img: Image.Image, **kw):
    b = io.BytesIO()
    img.save(b, format="PNG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "P"])
@pytest.mark.parametrize("shape", [(1, 1), (3, 17), (64, 72), (37, 129)])
@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_pil_written_pngs(mode, shape, level, tmp_path):
    rng = np.random.default_rng(hash((mode, shape, level)) & 0xffff)
    H, W = shape
    y, x = np.mgrid[0:H, 0:W]
    smooth = np.stack([(x * 3 + y * (c + 1)) % 256 for c in range(4)], -1).astype(np.uint8)
    noise = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    arr = np.where(rng.random((H, W, 1)) < 0.5, smooth, noise)
    if mode == "P":
        im = Image.fromarray(arr[..., :3]).quantize(colors=37)
    else:
        im = Image.fromarray(arr[..., :len(mode)] if mode not in ("L",) else arr[..., 0], mode=mode)
    png = _pil_png(im, compress_level=level)
    got = _native(png, tmp_path)
    assert got is not None
    assert np.array_equal(got, _pil_rgb(png))


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xffffffff)


def _write_png(arr: np.ndarray, filters, idat_split=1):
    """Test-only PNG writer: RGB 8-bit, scanline filter filters[y % len]."""
    H, W, C = arr.shape
    bpp, ctype = C, {1: 0, 2: 4, 3: 2, 4: 6}[C]
    a = arr.reshape(H, W * C).astype(np.int32)
    raw = bytearray()
    for y in range(H):
        f = filters[y % len(filters)]
        cur = a[y]
        prev = a[y - 1] if y > 0 else np.zeros_like(cur)
        left = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        ul = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        if f == 0:
            out = cur
        elif f == 1:
            out = cur - left
        elif f == 2:
            out = cur - prev
        elif f == 3:
            out = cur - ((left + prev) >> 1)
        else:
            p = left + prev - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, ul))
            out = cur - pred
        raw += bytes([f]) + (out & 0xff).astype(np.uint8).tobytes()
    z = zlib.compress(bytes(raw), 6)
    parts = [z[i * len(z) // idat_split:(i + 1) * len(z) // idat_split] for i in range(idat_split)]
    ihdr = struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + b"".join(_chunk(b"IDAT", p) for p in parts) + \
        _chunk(b"IEND", b"")


@pytest.mark.parametrize("filters", [[0], [1], [2], [3], [4], [0, 1, 2, 3, 4], [4, 3, 2, 1]])
@pytest.mark.parametrize("C", [3, 4])
def test_every_filter_type(filters, C, tmp_path):
    rng = np.random.default_rng(C * 10 + len(filters))
    arr = rng.integers(0, 256, (23, 31, C), dtype=np.uint8)
    arr[5:15] = arr[5:6]          # repeated rows: the Up / Paeth paths see real predictions
    png = _write_png(arr, filters, idat_split=3)
    got = _native(png, tmp_path)
    assert np.array_equal(got, _pil_rgb(png))


def test_corrupt_png_raises(tmp_path):
    arr = np.random.default_rng(0).integers(0, 256, (8, 8, 3), dtype=np.uint8)
    png = bytearray(_write_png(arr, [1]))
    png[-20] ^= 0xFF              # inside the IDAT body: CRC mismatch
    with pytest.raises(ValueError):
        _native(bytes(png), tmp_path)
    with pytest.raises(ValueError):
        _native(bytes(_write_png(arr, [1]))[:60], tmp_path)


@pytest.mark.parametrize("C", [1, 2])
def test_gray_is_not_a_colour_frame(C, tmp_path):
    """Gray PNGs stay 2-D / 2-channel (the reference's cvtColor(BGR2RGB) rejects
    them), so encode_fn raises as it did with PIL reading them."""
    arr = np.random.default_rng(C).integers(0, 256, (9, 11, C), dtype=np.uint8)
    png = _write_png(arr, [0, 4])
    assert _native(png, tmp_path) is None
    p = tmp_path / "g.png"
    p.write_bytes(png)
    img, _ = eic.read_image(str(p))
    assert img.ndim == 2 or img.shape[2] != 3


def test_16bit_falls_back_to_pil(tmp_path):
    a = (np.arange(12 * 10, dtype=np.uint16).reshape(12, 10) * 97).astype(np.uint16)
    p = tmp_path / "g16.png"
    Image.fromarray(a).save(p)
    img, _ = eic._read_png_native(str(p))
    assert img is None                     # not covered natively
    got, _ = eic.read_image(str(p))        # PIL path
    assert got.shape[:2] == (12, 10)


def test_read_image_uses_native_reader(tmp_path):
    arr = np.random.default_rng(3).integers(0, 256, (40, 50, 3), dtype=np.uint8)
    p = tmp_path / "f.png"
    Image.fromarray(arr).save(p)
    got, n = eic.read_image(str(p))
    assert np.array_equal(got, arr) and n == p.stat().st_size


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (17, 1000), (600, 700), (1100, 1000)])
def test_png_writer_round_trip(shape, tmp_path):
    """eic.write_image's native writer (vcf_png_encode_rgb): PIL and the native
    reader read back the same pixels; the bytes do not depend on the thread
    count (fixed 1 MiB deflate pieces)."""
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    a = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    a[: shape[0] // 2] //= 16                 # some compressible rows
    outs = []
    for th in (1, 8):
        eic.PNG_THREADS = th
        p = tmp_path / f"w{th}.png"
        n = eic.write_image(str(p), a)
        assert n == p.stat().st_size
        assert np.array_equal(np.asarray(Image.open(p).convert("RGB")), a)
        assert np.array_equal(eic.read_image(str(p))[0], a)
        outs.append(p.read_bytes())
    eic.PNG_THREADS = 16
    assert outs[0] == outs[1]


def test_libdeflate_and_zlib_paths_agree(tmp_path):
    """The reader inflates with libdeflate when the system has it and with zlib
    otherwise (VCF_PNG_NO_LIBDEFLATE=1 forces zlib): same pixels, same errors."""
    import subprocess
    import sys
    rng = np.random.default_rng(5)
    files = []
    for n, (filters, split) in enumerate((([1, 2], 1), ([0, 1, 2, 3, 4], 4), ([4], 2))):
        arr = rng.integers(0, 256, (37, 29, 3), dtype=np.uint8)
        arr[10:20] = arr[10:11]
        p = tmp_path / f"f{n}.png"
        p.write_bytes(_write_png(arr, filters, idat_split=split))
        files.append(str(p))
    bad = tmp_path / "trailing.png"   # extra scanline data after the image: both paths take the first rows
    arr = rng.integers(0, 256, (6, 5, 3), dtype=np.uint8)
    png = _write_png(np.concatenate([arr, arr]), [1])
    ihdr = struct.pack(">IIBBBBB", 5, 6, 8, 2, 0, 0, 0)
    bad.write_bytes(png[:8] + _chunk(b"IHDR", ihdr) + png[8 + 25:])
    files.append(str(bad))
    code = ("import sys, numpy as np\nfrom vcf_amd.codec import eic\n"
            "np.savez(sys.argv[1], *[eic.read_image(f)[0] for f in sys.argv[2:]])\n")
    outs = []
    for flag in ("0", "1"):
        out = str(tmp_path / f"o{flag}.npz")
        env = dict(os.environ, VCF_PNG_NO_LIBDEFLATE=flag)
        subprocess.run([sys.executable, "-c", code, out, *files], check=True, env=env, cwd=ROOT)
        outs.append(np.load(out))
    for k in outs[0].files:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    for f, k in zip(files, outs[0].files):
        assert np.array_equal(outs[0][k], _pil_rgb(open(f, "rb").read())), f
