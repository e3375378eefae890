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


def test_tiff_strips_rejects_inconsistent_tables():
    """tiff_strips returns None (host reader) for a strip table the GPU inflate
    could not trust: an extra strip, a strip past the end of the file, and
    parses an IFD that lies beyond the first 64 KiB."""
    import struct

    import numpy as np

    from vcf_amd.codec.tiff import imwrite_bytes, tiff_strips
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (300, 300, 3), dtype=np.uint8)
    buf = imwrite_bytes(img)
    shape, dt, offs, counts, sb = tiff_strips(buf)
    assert shape == (300, 300, 3) and len(offs) == -(-img.nbytes // sb)

    def patched(new_offs, new_counts):
        # rebuild a minimal little-endian TIFF around the same strips with the given table
        n = len(new_offs)
        entries = [(256, 3, 1, 300), (257, 3, 1, 300), (258, 3, 1, 8), (259, 3, 1, 8), (262, 3, 1, 2),
                   (277, 3, 1, 3), (278, 3, 1, sb // 900), (284, 3, 1, 1)]
        data = bytearray(buf)
        arr_off = len(data)
        data += struct.pack("<%dI" % n, *new_offs)
        cnt_off = len(data)
        data += struct.pack("<%dI" % n, *new_counts)
        ifd_off = len(data)
        tags = sorted(entries + [(273, 4, n, arr_off if n > 1 else new_offs[0]),
                                 (279, 4, n, cnt_off if n > 1 else new_counts[0])])
        data += struct.pack("<H", len(tags))
        for code, typ, count, val in tags:
            data += struct.pack("<HHI", code, typ, count) + (struct.pack("<HH", val, 0) if typ == 3 and count == 1
                                                              else struct.pack("<I", val))
        data += struct.pack("<I", 0)
        data[4:8] = struct.pack("<I", ifd_off)
        return bytes(data)

    # the same table, IFD written at the end (past 64 KiB): parsed, same strips
    big = patched(offs, counts)
    assert ifd_beyond_small(big)
    got = tiff_strips(big)
    assert got is not None and got[2] == offs and got[3] == counts
    assert tiff_strips(patched(offs + [offs[-1]], counts + [counts[-1]])) is None   # an extra strip
    assert tiff_strips(patched(offs[:-1], counts[:-1])) is None                     # a missing strip
    bad = list(counts)
    bad[-1] = len(big) + 10
    assert tiff_strips(patched(offs, bad)) is None                                  # past the end of the file
    assert tiff_strips(b"II*\x00\xff\xff\x00\x00") is None                          # IFD offset out of range


def ifd_beyond_small(b):
    import struct
    return struct.unpack("<I", b[4:8])[0] >= 65536
