"""Host-side TIFF helpers the GPU paths build on (CPU only): the batched
container prefixes of the HBM-resident -c TIFF paths (DeviceIII / DeviceIPP)
and the strip table the GPU inflate reads (dct2d.decode_fns), against the
host writer and the reference's own .tif fixtures."""
import glob
import os
import zlib

import numpy as np
import pytest

from vcf_amd.codec.tiff import (container_prefix, container_prefixes, imread_bytes, imwrite_bytes, strip_layout,
                                tiff_strips)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("shape,dtype", [((1080, 1920, 3), np.uint8), ((40, 48, 3), np.uint8),
                                         ((33, 70), np.uint16), ((2160, 3840, 3), np.uint8)])
def test_container_prefixes_equal_per_frame_prefix(shape, dtype):
    C = shape[2] if len(shape) > 2 else 1
    ns = strip_layout((shape[0], shape[1], C), np.dtype(dtype).itemsize)[1]
    rng = np.random.default_rng(ns)
    counts = rng.integers(1, 70000, (5, ns))
    rows = container_prefixes(shape, dtype, counts)
    for f in range(5):
        assert rows[f].tobytes() == container_prefix(shape, dtype, counts[f].tolist())


@pytest.mark.parametrize("shape,dtype", [((72, 96, 3), np.uint8), ((1080, 1920, 3), np.uint8),
                                         ((50, 60), np.uint16), ((7, 5, 3), np.uint16)])
def test_tiff_strips_of_host_files(shape, dtype):
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 200, shape).astype(dtype)
    buf = imwrite_bytes(img)
    got = tiff_strips(buf)
    assert got is not None
    shp, dt, offs, counts, sbytes = got
    assert tuple(shp) == shape and dt == np.dtype(dtype)
    raw = b"".join(zlib.decompress(buf[o:o + c]) for o, c in zip(offs, counts))
    assert raw == img.astype(dt).tobytes()
    assert all(len(zlib.decompress(buf[o:o + c])) == sbytes for o, c in zip(offs[:-1], counts[:-1]))


def test_tiff_strips_of_reference_files():
    """The reference's own .tif files (tifffile 2021.7.2 via TIFF.py:29) parse to
    strips that inflate to the fixture's indices."""
    files = sorted(glob.glob(os.path.join(GOLDEN, "dct_*.npz")))
    n = 0
    for fn in files:
        with np.load(fn, allow_pickle=False) as z:
            if "tif" not in z.files or "k" not in z.files:
                continue
            tif, k = z["tif"].tobytes(), z["k"]
        got = tiff_strips(tif)
        assert got is not None, fn
        shp, dt, offs, counts, _ = got
        raw = b"".join(zlib.decompress(tif[o:o + c]) for o, c in zip(offs, counts))
        assert raw == np.ascontiguousarray(k).astype(dt).tobytes(), fn
        assert np.array_equal(imread_bytes(tif), k), fn
        n += 1
    assert n > 0
