"""TIFF entropy stage (src/TIFF.py) on the CPU: the writer reproduces the
reference's .tif files byte for byte (tifffile 2021.7.2, zlib level 6); the
reader decodes them and the imagecodecs/libdeflate variant."""
import hashlib
import importlib.util
import io
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases, load_case
from vcf_amd.codec.tiff import TIFFCodec, imread_bytes, imwrite_bytes


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_tiff_bytes_equal_reference(case):
    d = load_case(case)
    assert imwrite_bytes(d["k"]) == bytes(d["tif"])
    assert case["encode_bytes"] == len(d["tif"])


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_tiff_reader(case):
    d = load_case(case)
    assert np.array_equal(imread_bytes(bytes(d["tif"])), d["k"])
    if "tif_libdeflate" in d.files:
        assert np.array_equal(imread_bytes(bytes(d["tif_libdeflate"])), d["k"])


def test_tiff_multi_strip_512_cases(manifest):
    """512x512x3 u8 -> RowsPerStrip 42, 13 strips (config C1); SHA-256 of the
    reference's file, from indices the golden-pinned oracle produces."""
    from oracle import oracle as O
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    for case in manifest["big_cases"]:
        rgb = m.synth(case["kind"], case["H"], case["W"], case["seed"])
        t = imwrite_bytes(O.encode_frame(rgb, 32, 0))
        assert len(t) == case["encode_bytes"]
        assert hashlib.sha256(t).hexdigest() == case["sha256"]["tif"]


def test_tiff_strip_layout_1080p():
    """1080p: RowsPerStrip = 65536 // 5760 = 11 -> 99 strips."""
    k = np.random.Generator(np.random.PCG64(5)).integers(0, 4, (1080, 1920, 3), dtype=np.uint8)
    t = imwrite_bytes(k)
    n = struct.unpack("<H", t[8:10])[0]
    ent = {}
    for i in range(n):
        code, typ, count, value = struct.unpack("<HHII", t[10 + 12 * i:22 + 12 * i])
        ent[code] = (count, value)
    assert ent[278] == (1, 11)                         # RowsPerStrip
    assert ent[273][0] == 99 and ent[279][0] == 99     # StripOffsets / StripByteCounts
    assert np.array_equal(imread_bytes(t), k)


def test_tiff_uint16_and_codec_surface():
    a = np.arange(24 * 16 * 3, dtype=np.uint16).reshape(24, 16, 3) * 97
    c = TIFFCodec()
    b = c.compress(a)
    assert isinstance(b, io.BytesIO) and b.tell() == 0
    assert np.array_equal(c.decompress(b.read()), a)
    assert c.file_extension == ".tif"
    with pytest.raises(AssertionError):
        c.compress(a.astype(np.float32))


def _dwt_cases():
    import json
    return json.load(open(os.path.join(GOLDEN, "manifest_dwt.json")))["cases"]


@pytest.mark.parametrize("case", _dwt_cases(), ids=lambda c: c["name"])
def test_tiff_dwt_subband_files_equal_reference(case):
    """2D-DWT.py:162-200 writes LL as uint16 and details as uint8 TIFFs."""
    d = np.load(os.path.join(GOLDEN, f"dwt_{case['name']}.npz"))
    L = case["levels"]
    assert imwrite_bytes(d[f"LL_{L}"]) == bytes(d["tif_LL"])
    assert imwrite_bytes(d["HH_1"]) == bytes(d["tif_HH_1"])
    assert np.array_equal(imread_bytes(bytes(d["tif_LL"])), d[f"LL_{L}"])
