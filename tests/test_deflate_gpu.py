"""GPU TIFF strip deflate (vcf_zlib_strips, csrc/vcf_deflate.hip) against
zlib.compress, byte for byte, and the TIFF files around the strips against the
host writer (the reference's TIFF.py:29 via tifffile -> zlib level 6)."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(n, shape, seed, kind="image"):
    rng = np.random.default_rng(seed)
    out = []
    for f in range(n):
        if kind == "image":
            H, W, C = shape
            y = np.arange(H)[:, None, None]
            x = np.arange(W)[None, :, None]
            a = 128 + 60 * np.sin(x / (37 + f) + np.arange(C)) + 50 * np.cos(y / 23.0 - f) + rng.normal(0, 4, shape)
            out.append(np.clip(a, 0, 255).astype(np.uint8))
        elif kind == "random":
            out.append(rng.integers(0, 256, shape, dtype=np.uint8))
        else:   # DCT-index-like: mostly 128 with sparse values
            a = np.full(shape, 128, np.uint8)
            m = rng.random(shape) < 0.03
            a[m] = rng.integers(100, 160, int(m.sum()))
            out.append(a)
    return np.stack(out)


def _check(frames, strip_bytes, level=6):
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import StripDeflater
    n = frames.shape[0]
    flat = frames.reshape(n, -1)
    d = DeviceBuffer.from_array(flat)
    got = StripDeflater().deflate_device(d, n, flat.shape[1], strip_bytes, level)
    for f in range(n):
        b = flat[f].tobytes()
        want = [zlib.compress(b[i:i + strip_bytes], level) for i in range(0, len(b), strip_bytes)]
        assert len(got[f]) == len(want)
        for k, (g, w) in enumerate(zip(got[f], want)):
            assert g == w, (f, k, len(g), len(w))


@pytest.mark.parametrize("kind", ["image", "random", "sparse"])
def test_strips_equal_zlib(kind):
    _check(_frames(3, (40, 300, 3), 1, kind), 11 * 900)


@pytest.mark.parametrize("strip", [65536, 65300, 65280, 65274, 1, 2, 3, 258, 4096])
def test_strip_lengths(strip):
    _check(_frames(2, (48, 700, 3), 2, "image"), strip)


def test_slide_nil_head():
    """zlib's slide_hash maps the head entry at input position wsize to NIL
    (tests/deflate_cases.py): the GPU must emit zlib's literal there."""
    from deflate_cases import slide_nil_strip
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import StripDeflater
    b = np.frombuffer(slide_nil_strip(), np.uint8)
    frames = np.stack([b, b[::-1].copy()])
    d = DeviceBuffer.from_array(frames)
    for level in (4, 6, 9):
        got = StripDeflater().deflate_device(d, 2, b.size, b.size, level)
        assert got[0][0] == zlib.compress(b.tobytes(), level), level
        assert got[1][0] == zlib.compress(b[::-1].tobytes(), level), level


@pytest.mark.parametrize("level", [4, 5, 7, 8, 9])
def test_levels(level):
    _check(_frames(1, (30, 1000, 3), 3, "image"), 65536, level)


def test_1080p_dct_frame_equals_host_tiff():
    """A 1080p frame of DCT indices (the C2 path): the GPU TIFF equals the host writer's bytes."""
    from vcf_amd.synthetic import synth_frame
    from vcf_amd.codec.tiff import imwrite_bytes
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import tiff_frames_device
    from vcf_amd import dct
    rgb = np.stack([synth_frame(1080, 1920, s) for s in (1, 2)])
    k = dct.encode(rgb, Q=32)
    d = DeviceBuffer.from_array(np.ascontiguousarray(k))
    files = tiff_frames_device(d, 2, k.shape[1:], np.uint8)
    for f in range(2):
        assert files[f] == imwrite_bytes(k[f])


def test_u16_and_gray():
    from vcf_amd.codec.tiff import imwrite_bytes
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import tiff_frames_device
    rng = np.random.default_rng(5)
    a = (rng.integers(0, 600, (3, 70, 130, 3))).astype(np.uint16)
    files = tiff_frames_device(DeviceBuffer.from_array(a), 3, a.shape[1:], np.uint16)
    assert all(files[f] == imwrite_bytes(a[f]) for f in range(3))
    g = rng.integers(120, 136, (2, 300, 333), dtype=np.uint8)
    files = tiff_frames_device(DeviceBuffer.from_array(g), 2, g.shape[1:], np.uint8)
    assert all(files[f] == imwrite_bytes(g[f]) for f in range(2))


def test_unsupported():
    from vcf_amd import _lib as L
    from vcf_amd.device import DeviceBuffer
    d = DeviceBuffer(1 << 20)
    for level, strip in ((1, 4096), (6, 65537), (0, 4096)):
        with pytest.raises(Exception):
            L.call("vcf_zlib_strips", d.ptr, 1, 8192, strip, level, d.ptr, 1 << 17, d.ptr, d.ptr, None)


def test_device_iii_tiff_equals_host_writer():
    """The C4 data path with the reference's default -c TIFF
    (vcf_amd/codec/iii_device.py, entropy="TIFF"): every gathered file equals
    the host TIFF writer's (system zlib) for the frame's indices, and reads back."""
    from vcf_amd.codec.iii_device import DeviceIII
    from vcf_amd.codec.tiff import imread_bytes, imwrite_bytes
    from vcf_amd import dct
    from vcf_amd.device import DeviceBuffer
    rng = np.random.default_rng(3)
    for n, H, W in ((5, 61, 77), (3, 200, 1000)):
        y = np.arange(H)[:, None, None]
        x = np.arange(W)[None, :, None]
        frames = np.stack([np.clip(128 + 50 * np.sin(x / (19 + f) + y / 31.0 + np.arange(3)) +
                                   rng.normal(0, 6, (H, W, 3)), 0, 255).astype(np.uint8) for f in range(n)])
        job = DeviceIII(None, 0, 1, n, H, W, 32, entropy="TIFF")
        stages = {}
        sizes, got = job.run(DeviceBuffer.from_array(frames), stages)
        k = dct.encode(frames, Q=32)
        for i in range(n):
            want = imwrite_bytes(k[i])
            assert got[i] == want and sizes[i] == len(want), (n, i)
            assert np.array_equal(imread_bytes(bytes(got[i])), k[i])


def _golden_tif_cases():
    import glob
    import os
    from conftest import GOLDEN
    return sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "dct_*.npz")))


@pytest.mark.parametrize("name", _golden_tif_cases())
def test_gpu_tiff_equals_reference_files(name):
    """The GPU deflate pinned to the reference's own bytes: the
    TIFF of every golden case's index array `k`, deflated on the GPU
    (tiff_frames_device), equals the .tif the reference's 2D-DCT.py wrote
    (tests/golden/dct_*.npz 'tif', tifffile 2021.7.2 + zlib, make_golden*.py)."""
    import os
    from conftest import GOLDEN
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import covers, tiff_frames_device
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    k = np.ascontiguousarray(z["k"])
    if k.dtype not in (np.uint8, np.uint16) or not covers(k.shape, k.dtype.itemsize):
        pytest.skip(f"{k.dtype} {k.shape}: not a TIFF the GPU deflate covers")
    files = tiff_frames_device(DeviceBuffer.from_array(k), 1, k.shape, k.dtype)
    assert files[0] == z["tif"].tobytes()


@pytest.mark.parametrize("name", ["smooth_512x512", "rand_512x512"])
def test_gpu_tiff_512_matches_reference_sha256(manifest, name):
    """The C1 cases by SHA-256 (tests/golden/manifest.json big_cases): the GPU
    deflate of the indices gives the reference's .tif."""
    import hashlib
    import importlib.util
    import os
    from conftest import GOLDEN
    from vcf_amd import dct
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import tiff_frames_device
    case = [c for c in manifest["big_cases"] if c["name"] == name][0]
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rgb = m.synth(case["kind"], case["H"], case["W"], case["seed"])
    k = dct.encode(rgb, Q=32)
    tif = tiff_frames_device(DeviceBuffer.from_array(np.ascontiguousarray(k)), 1, k.shape, np.uint8)[0]
    assert len(tif) == case["encode_bytes"]
    assert hashlib.sha256(tif).hexdigest() == case["sha256"]["tif"]


def test_c4_workload_every_strip_equals_zlib():
    """bench.py's C4 content (256 1080p DCT index frames, 25 344 strips): several
    workspace rounds, lazy and register-window strips side by side.  Every strip
    against zlib.compress: a strip coded from stale workspace data (the previous
    round's strip in the same slot) shows up here."""
    from concurrent.futures import ThreadPoolExecutor

    from vcf_amd import synthetic as bench
    from vcf_amd import dct
    from vcf_amd.codec.tiff import strip_layout
    from vcf_amd.device import DeviceBuffer
    from vcf_amd.zlib_gpu import StripDeflater
    n, H, W = 256, 1080, 1920
    bases = [bench.synth_frame(H, W, seed=100 + s) for s in range(4)]
    k = np.concatenate([dct.encode(np.stack([bench.c4_frame(bases, i) for i in range(f, f + 16)]), Q=32)
                        for f in range(0, n, 16)])
    flat = np.ascontiguousarray(k.reshape(n, -1))
    sb = strip_layout(k.shape[1:], 1)[2]
    got = StripDeflater().deflate_device(DeviceBuffer.from_array(flat), n, flat.shape[1], sb, 6)
    spf = len(got[0])
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda s: zlib.compress(flat[s // spf, (s % spf) * sb:(s % spf + 1) * sb].tobytes(), 6),
                           range(n * spf)))
    bad = [s for s in range(n * spf) if bytes(got[s // spf][s % spf]) != want[s]]
    assert not bad, bad[:20]


_MULTI_ROUND = r'''
import sys, zlib
import numpy as np
sys.path.insert(0, sys.argv[1])
from vcf_amd import synthetic as bench
from vcf_amd import dct
from vcf_amd import _lib as L
from vcf_amd.codec.tiff import strip_layout
from vcf_amd.device import DeviceBuffer
from vcf_amd.zlib_gpu import StripDeflater
n, H, W = 24, 1080, 1920
bases = [bench.synth_frame(H, W, seed=100 + s) for s in range(4)]
k = np.concatenate([dct.encode(np.stack([bench.c4_frame(bases, i) for i in range(f, f + 8)]), Q=32)
                    for f in range(0, n, 8)])
flat = np.ascontiguousarray(k.reshape(n, -1))
sb = strip_layout(k.shape[1:], 1)[2]
total = n * int(L.lib().vcf_zlib_strip_count(flat.shape[1], sb))
per = int(L.lib().vcf_zlib_workspace(total)) // (int(L.lib().vcf_zlib_workspace(1)))
got = StripDeflater().deflate_device(DeviceBuffer.from_array(flat), n, flat.shape[1], sb, 6)
spf = len(got[0])
bad = [s for s in range(n * spf)
       if bytes(got[s // spf][s % spf]) != zlib.compress(flat[s // spf, (s % spf) * sb:(s % spf + 1) * sb].tobytes(), 6)]
print("strips", total, "per_round", per, "bad", len(bad))
assert per < total and not bad, bad[:20]
'''


def test_many_rounds_every_strip_equals_zlib():
    """Deterministic multi-round run: the workspace budget forced down to ~50 MB
    (VCF_ZX_BUDGET, read once per process, so a child process) cuts 2 376 C4
    strips into rounds of 43 that reuse one workspace; every strip against
    zlib.compress (a strip coded from the previous round's tables shows here)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, VCF_ZX_BUDGET="50000000")
    p = subprocess.run([sys.executable, "-c", _MULTI_ROUND, root], env=env, capture_output=True, text=True,
                       timeout=280)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "bad 0" in p.stdout
