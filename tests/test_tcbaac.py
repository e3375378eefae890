"""Tiled CBAAC container (vcf_amd/tcbaac.py) on the host: layout, index
checks and the reference's malformed-header behaviour (CBAAC.py:101-102).
The coding itself runs on the GPU (tests/test_tcbaac_gpu.py)."""
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
                                 T.pack((4, 4), 0, 256, [3], b"abc").replace(b"VCFT", b"XXXX")])
def test_malformed_streams_decode_to_reference_zeros(bad):
    assert np.array_equal(T.TiledCBAACCodec().decompress(bad), np.zeros((10, 10), np.uint8))


def test_segment_count():
    assert T.n_segments(0, 256) == 0
    assert T.n_segments(1, 256) == 1
    assert T.n_segments(1080 * 1920 * 3, T.DEFAULT_SEG) == 48
    assert T.n_segments(2160 * 3840 * 3, T.DEFAULT_SEG) == 190
