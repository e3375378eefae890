"""Tiled CBAAC container (vcf_amd/tcbaac.py) on the host: layout, index
checks and the reference's malformed-header behaviour (CBAAC.py:101-102).
The coding itself runs on the GPU (tests/test_tcbaac_gpu.py)."""
import struct

import numpy as np
import pytest

from vcf_amd import tcbaac as T


def test_container_round_trip_and_layout():
    sizes = np.array([5, 0, 7], np.int64)
    payload = bytes(range(12))
    data = T.pack((2, 100, 3), 1, 256, sizes, payload)
    assert data[:16] == np.array([3, 2, 100, 3], np.uint32).tobytes()     # CBAAC.py:84-89 fields first
    assert data[16:20] == b"VCFT"
    shape, order, seg_len, sb, pl = T.unpack(data)
    assert shape == (2, 100, 3) and order == 1 and seg_len == 256
    assert list(sb) == [5, 0, 7] and pl == payload


@pytest.mark.parametrize("bad", [b"\x01", b"", T.pack((4, 4), 0, 256, [3], b"abc")[:-1],
                                 T.pack((4, 4), 0, 256, [3], b"abc").replace(b"VCFT", b"XXXX"),
                                 # version-1 headers the GPU coder cannot take: order > 1,
                                 # a segment length that is not a positive multiple of 256
                                 T.pack((4, 4), 2, 256, [3], b"abc"),
                                 T.pack((4, 4), 0, 300, [3], b"abc"),
                                 T.pack((4, 4), 0, 0, [3], b"abc")])
def test_malformed_streams_decode_to_reference_zeros(bad):
    assert np.array_equal(T.TiledCBAACCodec().decompress(bad), np.zeros((10, 10), np.uint8))


def test_segment_count():
    assert T.n_segments(0, 256) == 0
    assert T.n_segments(1, 256) == 1
    assert T.n_segments(1080 * 1920 * 3, T.DEFAULT_SEG) == 48
    assert T.n_segments(2160 * 3840 * 3, T.DEFAULT_SEG) == 190


def test_container_version_2_carries_the_prior():
    prior = (np.arange(256) % 50 + 1).astype(np.uint16)
    data = T.pack((4, 70), 0, 256, [3, 2], b"abcde", prior)
    assert struct.unpack_from("<I", data, 16)[0] == T.VERSION_PRIOR
    shape, order, seg_len, sb, pl, pr = T._parse(data)
    assert shape == (4, 70) and list(sb) == [3, 2] and pl == b"abcde" and np.array_equal(pr, prior)
    assert T.unpack(data)[:3] == ((4, 70), 0, 256)
    with pytest.raises(ValueError):
        T.pack((4, 70), 0, 256, [3, 2], b"abcde", np.zeros(256, np.uint16))    # a zero frequency
    with pytest.raises(ValueError):
        T.pack((4, 70), 0, 256, [3, 2], b"abcde", np.full(256, 64, np.uint16))  # total >= max_freq


def test_prior_formula():
    sym = np.array([0] * 900 + [5] * 90 + [255] * 10, np.uint8)
    p = T.prior_of(sym)
    assert p[0] == 1 + 900 * 8192 // 1000 and p[5] == 1 + 90 * 8192 // 1000 and p[255] == 1 + 10 * 8192 // 1000
    assert p[1] == 1 and int(p.sum()) < 16384
    assert np.array_equal(T.prior_of(np.zeros(0, np.uint8)), np.ones(256, np.uint16))


def test_host_coder_with_prior():
    """vcf_cbaac_encode_prior: all-ones prior == the reference's model; a
    skewed prior round-trips and codes a skewed segment in fewer bytes."""
    rng = np.random.Generator(np.random.PCG64(4))
    sym = np.where(rng.random(20000) < 0.97, 128, rng.integers(0, 256, 20000)).astype(np.uint8)
    ones = np.ones(256, np.uint16)
    assert T.host_segments_prior(sym, ones, 4096) == T.host_segments(sym, 0, 4096)
    p = T.prior_of(sym)
    segs = T.host_segments_prior(sym, p, 4096)
    assert sum(map(len, segs)) < sum(map(len, T.host_segments(sym, 0, 4096)))
    for i, s in enumerate(segs):
        part = sym[i * 4096:(i + 1) * 4096]
        assert np.array_equal(T.host_decode_prior(s, part.size, p), part)
    assert T.host_segments_prior(sym, ones, 4096, 1) == T.host_segments(sym, 1, 4096)   # order 1, all contexts
    for i, s in enumerate(T.host_segments_prior(sym, p, 4096, 1)):
        part = sym[i * 4096:(i + 1) * 4096]
        assert np.array_equal(T.host_decode_prior(s, part.size, p, 1), part)


def test_prior_codec_is_registered():
    from vcf_amd.codec.dct2d import ENTROPY_CODECS
    c = ENTROPY_CODECS["TCBAACP"]()
    assert c.prior and c.ORDER == 0 and c.file_extension == ".tadpt_arith"
    assert c.seg_len == T.CLASS_SEG and c.nclass == T.PRIOR_CLASSES


def test_container_version_3_carries_sparse_prior_rows():
    """Version 3: nclass prior rows stored sparsely (only the frequencies != 1)."""
    rows = np.ones((5, 256), np.uint16)
    rows[0, [0, 128, 255]] = [7, 8000, 2]
    rows[3, 128] = 8193
    data = T.pack((4, 70), 0, 256, [3, 2], b"abcde", rows)
    assert struct.unpack_from("<I", data, 16)[0] == T.VERSION_CLASSES
    shape, order, seg_len, sb, pl, pr = T._parse(data)
    assert shape == (4, 70) and list(sb) == [3, 2] and pl == b"abcde" and np.array_equal(pr, rows)
    assert len(data) == 12 + 4 + 16 + 4 + 5 * 2 + 4 * 3 + 2 + 5   # shape, magic, fields, nclass, rows, varint sizes, payload
    with pytest.raises(ValueError):
        T.pack((4, 70), 0, 256, [3, 2], b"abcde", np.full((2, 256), 64, np.uint16))
    bad = bytearray(data)
    struct.pack_into("<I", bad, 32, 0)   # zero classes
    assert np.array_equal(T.TiledCBAACCodec().decompress(bytes(bad)), np.zeros((10, 10), np.uint8))


def test_class_prior_formula():
    """prior_of(sym, nclass, seg_len): row c over the symbols of the segments s
    with s * nclass // n_segments == c; rows without segments stay ones."""
    sym = np.concatenate([np.zeros(1000, np.uint8), np.full(1000, 9, np.uint8), np.full(560, 3, np.uint8)])
    rows = T.prior_of(sym, 3, 256)          # 10 segments: classes 0-3, 4-6, 7-9
    assert rows.shape == (3, 256)
    assert np.array_equal(rows[0], T.prior_of(sym[:1024]))
    assert np.array_equal(rows[1], T.prior_of(sym[1024:1792]))
    assert np.array_equal(rows[2], T.prior_of(sym[1792:]))
    few = T.prior_of(sym[:300], 4, 256)      # 2 segments, 4 classes: rows 1 and 3 unused
    assert np.array_equal(few[1], np.ones(256, np.uint16)) and np.array_equal(few[3], np.ones(256, np.uint16))
    assert np.array_equal(few[0], T.prior_of(sym[:256])) and np.array_equal(few[2], T.prior_of(sym[256:300]))


def test_version_3_segment_index_varints():
    """The version-3 segment sizes are LEB128 varints: 1 byte below 128, up to
    5 bytes; truncated or overlong indexes are malformed."""
    sizes = np.array([0, 1, 127, 128, 300, 16383, 16384, 2 ** 21, 2 ** 28 + 5, 2 ** 32 - 1], np.int64)
    enc = T._varints(sizes)
    assert len(enc) == 1 + 1 + 1 + 2 + 2 + 2 + 3 + 4 + 5 + 5
    got, end = T._parse_varints(enc + b"xyz", 0, sizes.size)
    assert list(got) == list(sizes) and end == len(enc)
    with pytest.raises(ValueError):
        T._parse_varints(enc[:-1], 0, sizes.size)
    with pytest.raises(ValueError):
        T._parse_varints(b"\x80" * 6 + b"\x01", 0, 1)
    rows = np.ones((2, 256), np.uint16)
    n = 256 * 40
    segs = np.arange(40) * 7 % 300
    data = T.pack((n,), 0, 256, segs, bytes(int(segs.sum())), rows)
    assert list(T._parse(data)[3]) == list(segs)