"""CBAAC (src/CBAAC.py) on the host: the native model reproduces the
reference's own AdaptiveModel/ContextManager step for step (traces made by
executing the reference's classes, tests/golden/make_golden_cbaac.py), and
the A8 arithmetic coder round-trips exactly.  The coder's bytes are parity
unpinned: the reference's coder package (arithmetic_coding) is not vendored
and its outputs are not in the tree."""
import io
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from vcf_amd import cbaac as C

_MAN = json.load(open(os.path.join(GOLDEN, "manifest_cbaac.json")))


@pytest.mark.parametrize("case", _MAN["cases"], ids=lambda c: f"{c['stream']}_o{c['order']}")
def test_model_trace_equals_reference(case):
    d = np.load(os.path.join(GOLDEN, "cbaac_model.npz"))
    sym = d[f"sym_{case['stream']}"]
    ref = d[f"trace_{case['stream']}_o{case['order']}"]
    got = C.model_trace(sym, case["order"])
    bad = np.nonzero(np.any(got != ref, axis=1))[0]
    assert bad.size == 0, (bad[:5], got[bad[:3]], ref[bad[:3]])


@pytest.mark.parametrize("order", [0, 1, 2, 3, 8])
def test_round_trip(order):
    rng = np.random.Generator(np.random.PCG64(order))
    for sym in (np.clip(np.rint(rng.laplace(128, 2, 50000)), 0, 255).astype(np.uint8),
                rng.integers(0, 256, 20000, dtype=np.uint8),
                np.full(30000, 7, np.uint8),
                np.array([255], np.uint8),
                np.zeros(0, np.uint8)):
        data = C.encode_symbols(sym, order)
        assert np.array_equal(C.decode_symbols(data, sym.size, order), sym)


def test_rate_is_near_entropy():
    rng = np.random.Generator(np.random.PCG64(9))
    sym = np.clip(np.rint(rng.laplace(128, 2, 200000)), 0, 255).astype(np.uint8)
    p = np.bincount(sym, minlength=256) / sym.size
    H = -np.sum(p[p > 0] * np.log2(p[p > 0]))
    bits = 8 * len(C.encode_symbols(sym, 0))
    assert bits / sym.size < H * 1.02 + 0.01


def test_container_matches_reference_layout():
    """uint32 ndims, uint32 shape (CBAAC.py:84-89), then the bit stream."""
    img = np.random.Generator(np.random.PCG64(1)).integers(120, 136, (5, 7, 3), dtype=np.uint8)
    c = C.CBAACCodec(order=1)
    b = c.compress(img)
    raw = b.getvalue()
    assert raw[:4] == np.uint32(3).tobytes() and raw[4:16] == np.array([5, 7, 3], np.uint32).tobytes()
    assert raw[16:] == C.encode_symbols(img, 1)
    assert np.array_equal(c.decompress(raw), img)
    assert c.decompress(b"\x01").shape == (10, 10)          # CBAAC.py:101-102
    assert c.file_extension == ".adpt_arith"


def test_errors():
    with pytest.raises(ValueError):
        C.encode_symbols(np.zeros(4, np.uint8), 9)
    with pytest.raises(ValueError):
        C.CBAACCodec().compress(np.array([300], np.int32))


class _RefModel:
    """CBAAC.py:17-47's AdaptiveModel restated (its traces are pinned above):
    256 ones, +1 per update, halve (f >> 1) + 1 when the stale total >= 16384."""

    def __init__(self):
        self.freq = [1] * 256
        self.total = 256

    def _cum(self, s):
        return sum(self.freq[:s])

    def get_range(self, s):
        lo = self._cum(s)
        return lo, lo + self.freq[s], self.total

    def get_symbol_from_scaled_value(self, v):
        acc = 0
        for s, f in enumerate(self.freq):
            if acc + f > v:
                return s, acc, acc + f
            acc += f

    def update(self, s):
        stale = self.total
        self.freq[s] += 1
        if stale >= 16384:
            self.freq = [(f >> 1) + 1 for f in self.freq]
        self.total = sum(self.freq)


def _a8_encode(sym):
    import sys
    sys.path.insert(0, os.path.join(GOLDEN, "shims"))
    from arithmetic_coding.arithmetic_coding import Arithmetic_Encoding
    m, enc, bits = _RefModel(), Arithmetic_Encoding(), []
    for s in sym.tolist():
        enc.encode_symbol(s, m, bits)
        m.update(s)
    enc.flush(bits)
    bits += [0] * (-len(bits) % 8)
    return np.packbits(np.array(bits, np.uint8)).tobytes()


@pytest.mark.parametrize("kind", ["skewed", "uniform", "two_level", "rescales"])
def test_native_bytes_equal_a8_stand_in(kind):
    """The native coder (bulk renormalisation, reciprocal division, held-back
    MPS counts) writes exactly the bytes of A8 as the stand-in states it
    symbol by symbol: pending-bit runs, E1/E2 prefixes and rescales included."""
    rng = np.random.Generator(np.random.PCG64(21))
    sym = {"skewed": np.where(rng.random(6000) < 0.02, rng.integers(0, 256, 6000), 128),
           "uniform": rng.integers(0, 256, 3000),
           "two_level": np.where(rng.random(6000) < 0.5, 127, 128),
           "rescales": np.clip(np.rint(rng.laplace(128, 3, 40000)), 0, 255)}[kind].astype(np.uint8)
    got = C.encode_symbols(sym, 0)
    assert got == _a8_encode(sym)
    assert np.array_equal(C.decode_symbols(got, sym.size, 0), sym)
