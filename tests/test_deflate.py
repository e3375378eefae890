"""The GPU deflate's restatement of zlib (vcf_amd/csrc/vcf_deflate.h), built
for the host with a sequential hash-chain matcher (tests/cpu/deflate_harness.cpp),
against zlib.compress itself -- the oracle of TIFF.py:29's strips (tifffile ->
zlib level 6).  CPU only; the GPU kernel is tests/test_deflate_gpu.py."""
import ctypes
import os
import shutil
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpu", "deflate_harness.cpp")


@pytest.fixture(scope="module")
def dh(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    so = str(tmp_path_factory.mktemp("dh") / "deflate_harness.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(ROOT, "vcf_amd", "csrc"),
                    SRC, "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.dh_compress.restype = ctypes.c_longlong
    lib.dh_compress.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_char_p, ctypes.c_longlong]

    def compress(b: bytes, level: int = 6) -> bytes:
        out = ctypes.create_string_buffer(len(b) + len(b) // 8 + 1024)
        r = lib.dh_compress(b, len(b), level, out, len(out))
        assert r >= 0, r
        return out.raw[:r]
    return compress


def _cases():
    rng = np.random.default_rng(0)
    img = np.clip(128 + 40 * np.sin(np.arange(64 * 1100 * 3) / 300.0) + rng.normal(0, 3, 64 * 1100 * 3), 0, 255)
    img = img.astype(np.uint8).tobytes()
    runs = bytearray()
    while len(runs) < 65536:
        runs += bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 300))
    p = 0.5 ** np.arange(1, 33)
    return {
        "empty": b"", "one": b"\x80", "two": b"ab", "three": b"abc", "flat": b"\x80" * 5000,
        "random": rng.integers(0, 256, 40000, dtype=np.uint8).tobytes(),
        "alphabet4": rng.integers(0, 4, 60000, dtype=np.uint8).tobytes(),
        "text": (b"the quick brown fox jumps over the lazy dog " * 2000)[:65536],
        "runs": bytes(runs[:65536]),
        # skewed symbol distribution: Huffman lengths past 15 bits (gen_bitlen's overflow fix-up)
        "skewed": rng.choice(np.arange(32, dtype=np.uint8), 65536, p=p / p.sum()).tobytes(),
        "image_65536": img[:65536], "image_65300": img[:65300], "image_63360": img[:63360],
        # past wsize + MAX_DIST: zlib's window slides once and its stale bytes follow the end
        "zeros_65536": bytes(65536), "zeros_65280": bytes(65280), "random_65536": rng.integers(
            0, 256, 65536, dtype=np.uint8).tobytes(),
    }


def test_harness_slide_nil_head(dh):
    """slide_hash's NIL mapping of the head entry at input position wsize
    (ADVICE round 3): zlib writes a literal at strstart 65274 there."""
    from deflate_cases import slide_nil_strip
    b = slide_nil_strip()
    for level in (4, 5, 6, 7, 8, 9):
        assert dh(b, level) == zlib.compress(b, level), level


@pytest.mark.parametrize("level", [6, 4, 5, 7, 8, 9])
def test_harness_equals_zlib(dh, level):
    for name, b in _cases().items():
        assert dh(b, level) == zlib.compress(b, level), (name, level)


def test_harness_equals_zlib_fuzz(dh):
    rng = np.random.default_rng(7)
    for it in range(120):
        n = int(rng.choice([rng.integers(0, 400), rng.integers(0, 65537), rng.integers(65270, 65537)]))
        kind = it % 4
        if kind == 0:
            b = rng.integers(0, int(rng.integers(1, 256)), n, dtype=np.uint8).tobytes()
        elif kind == 1:
            ph = rng.integers(0, 256, int(rng.integers(3, 3000)), dtype=np.uint8)
            a = np.resize(ph, n).copy()
            m = rng.random(n) < rng.random() * 0.05
            a[m] = rng.integers(0, 256, int(m.sum()))
            b = a.tobytes()
        elif kind == 2:
            b = (128 + rng.integers(-2, 3, n)).astype(np.uint8).tobytes()
        else:
            b = np.repeat(rng.integers(0, 256, n // 50 + 1, dtype=np.uint8), 50)[:n].tobytes()
        level = int(rng.choice([6, 6, 4, 5, 7, 8, 9]))
        assert dh(b, level) == zlib.compress(b, level), (it, n, level)


@pytest.mark.parametrize("case", range(5))
def test_zlib_rejects_corrupt_code_lengths(case):
    """The oracle side of tests/test_inflate_gpu.py::test_rejects_corrupt_code_lengths:
    zlib.decompress rejects each hand-built stream with the named message."""
    from deflate_corrupt import CASES
    name, stream, msg, _ = CASES[case]
    with pytest.raises(zlib.error, match=msg):
        zlib.decompress(stream)
