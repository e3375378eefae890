"""CPU check of the HIP kernels' per-block arithmetic (vcf_dct_block.h, built
for the host with g++ -ffp-contract=off) against the oracle, bit for bit."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle import oracle as O

HARNESS_SRC = os.path.join(ROOT, "tests", "cpu", "block_harness.cpp")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    so = str(tmp_path_factory.mktemp("hb") / "block_harness.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", os.path.join(ROOT, "vcf_amd", "csrc"), HARNESS_SRC, "-o", so], check=True)
    L = ctypes.CDLL(so)
    u8 = ctypes.POINTER(ctypes.c_uint8)
    L.hb_encode_block.argtypes = [u8, ctypes.c_int, ctypes.c_uint, u8]
    L.hb_decode_block.argtypes = [u8, ctypes.c_int, ctypes.c_uint, u8]
    L.hb_encode_block_bytes.argtypes = [u8, ctypes.c_int, ctypes.c_uint, u8]
    L.hb_encode_block_cols.argtypes = [u8, ctypes.c_int, ctypes.c_uint, u8]
    L.hb_encode_block_fold.argtypes = [u8, ctypes.c_int, ctypes.c_uint, u8]
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


@pytest.mark.parametrize("Q,flags", [(32, 0), (7, 0), (1, 0), (64, 2), (5, 2), (3, 0), (1024, 0), (2, 2), (1 << 20, 0), (1 << 30, 2)])
def test_block_encode_decode_vs_oracle(harness, Q, flags):
    rng = np.random.Generator(np.random.PCG64(Q * 10 + flags))
    for it in range(300):
        if it % 3 == 0:
            blk = rng.integers(0, 256, (8, 8, 3), dtype=np.uint8)
        elif it % 3 == 1:
            blk = np.full((8, 8, 3), rng.integers(0, 256, 3), dtype=np.uint8)
        else:
            blk = (rng.integers(0, 2, (8, 8, 3)) * 255).astype(np.uint8)
        k = np.empty((8, 8, 3), np.uint8)
        harness.hb_encode_block(_p(blk), Q, flags, _p(k))
        kref = O.encode_frame(blk, Q, flags)
        assert np.array_equal(k, kref), (it, Q, flags)
        kb = np.empty((8, 8, 3), np.uint8)
        harness.hb_encode_block_bytes(_p(blk), Q, flags, _p(kb))
        assert np.array_equal(kb, kref), ("bytes", it, Q, flags)
        harness.hb_encode_block_cols(_p(blk), Q, flags, _p(kb))
        assert np.array_equal(kb, kref), ("cols", it, Q, flags)
        harness.hb_encode_block_fold(_p(blk), Q, flags, _p(kb))
        assert np.array_equal(kb, kref), ("fold", it, Q, flags)
        if Q > 32767:
            continue   # decode is int16 (A5): not defined past Q = 32767
        # decode arbitrary index blocks too (not only encoder outputs)
        kin = kref if it % 2 else rng.integers(0, 256, (8, 8, 3), dtype=np.uint8)
        out = np.empty((8, 8, 3), np.uint8)
        harness.hb_decode_block(_p(kin), Q, flags, _p(out))
        assert np.array_equal(out, O.decode_frame(kin, 8, 8, Q, flags)), (it, Q, flags)


def test_dct3_zero_skipping(harness):
    """dct3_8r_k<K> (inputs K..7 known zero) equals dct3_8r on such inputs: every
    nonzero output bit for bit, zeros equal up to their sign (the decode
    truncates to int16, where -0 and +0 are both 0)."""
    pd = ctypes.POINTER(ctypes.c_double)
    harness.hb_dct3.argtypes = [ctypes.c_int, pd, pd]
    rng = np.random.Generator(np.random.PCG64(3))
    for it in range(4000):
        K = int(rng.integers(1, 9))
        x = np.zeros(8)
        x[:K] = rng.integers(-2048, 2048, K) * rng.choice([1.0, 0.0625, 0.5])
        x[:K] *= rng.integers(0, 2, K)          # zeros inside the nonzero range too
        if it % 7 == 0:
            x[:K] = np.ldexp(rng.random(K) - 0.5, 20)   # the row pass takes non-integer inputs
        want, got = np.empty(8), np.empty(8)
        harness.hb_dct3(8, x.ctypes.data_as(pd), want.ctypes.data_as(pd))
        harness.hb_dct3(K, x.ctypes.data_as(pd), got.ctypes.data_as(pd))
        nz = (want != 0) | (got != 0)
        assert np.array_equal(want[nz].view(np.uint64), got[nz].view(np.uint64)), (K, x, want, got)
        assert np.array_equal(np.trunc(want), np.trunc(got))
