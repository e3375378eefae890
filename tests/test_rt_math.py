"""CPU check of the run-time-length block transforms the GPU kernels run
(vcf_pocketfft_rt.h + vcf_pocketfft_blue.h: rfftp with radfg/radbg, and the
Bluestein plans), built for the host (tests/cpu/rt_harness.hip, hipcc
--cuda-host-only -ffp-contract=off), against scipy's own outputs and the
oracle, bit for bit.  The plan building (rt_fill, blue_fill: twiddles, the
chirp bk and its transform bkf) is the same host code the library runs."""
import ctypes
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from oracle import oracle as O

SRC = os.path.join(ROOT, "tests", "cpu", "rt_harness.hip")


@pytest.fixture(scope="module")
def rt(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    so = str(tmp_path_factory.mktemp("rt") / "rt_harness.so")
    subprocess.run([hipcc, "--cuda-host-only", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", os.path.join(ROOT, "vcf_amd", "csrc"), "-I", os.path.join(ROOT, "include"), SRC, "-o", so],
                   check=True)
    L = ctypes.CDLL(so)
    for n in ("hb_rt_dct_f32", "hb_rt_dct_f64"):
        getattr(L, n).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.hb_rt_uses_bluestein.argtypes = [ctypes.c_int]
    L.hb_rt_n2.argtypes = [ctypes.c_int]
    return L


def _dct(L, kind, x, dtype):
    a = np.ascontiguousarray(np.array(x, dtype=dtype))
    N = a.shape[-1]
    f = L.hb_rt_dct_f32 if dtype == np.float32 else L.hb_rt_dct_f64
    assert f(kind, a.ctypes.data, N, a.size // N) == 0
    return a


BLUE = json.load(open(os.path.join(GOLDEN, "manifest_blue.json")))


def test_plan_choice_matches_pocketfft(rt):
    """pocketfft_r's Bluestein choice and good_size_cmplx, host vs oracle."""
    for N in range(1, 4097):
        assert bool(rt.hb_rt_uses_bluestein(N)) == O.dct_uses_bluestein(N), N
    assert [N for N in range(1, 601) if rt.hb_rt_uses_bluestein(N)] == BLUE["bluestein_lengths"]


def test_bluestein_blocks_vs_scipy(rt):
    """All 67 Bluestein lengths <= 600 against scipy.fftpack dct/idct (ortho)
    under the reference's python (make_golden_blue.py)."""
    g = np.load(os.path.join(GOLDEN, "blocks_blue.npz"))
    for N in BLUE["bluestein_lengths"]:
        fwd = _dct(rt, 2, g[f"fwd_in_{N}"], np.float32)
        assert np.array_equal(fwd.view(np.uint32), g[f"fwd_out_{N}"].view(np.uint32)), N
        inv = _dct(rt, 3, g[f"inv_in_{N}"].astype(np.float64), np.float64)
        assert np.array_equal(inv.view(np.uint64), g[f"inv_out_{N}"].view(np.uint64)), N


def test_rfftp_blocks_vs_scipy(rt):
    """The rfftp lengths (radfg/radbg included) of blocks_radg.npz."""
    radg = json.load(open(os.path.join(GOLDEN, "manifest_radg.json")))
    g = np.load(os.path.join(GOLDEN, "blocks_radg.npz"))
    for N in radg["lengths"]:
        fwd = _dct(rt, 2, g[f"fwd_in_{N}"], np.float32)
        assert np.array_equal(fwd.view(np.uint32), g[f"fwd_out_{N}"].view(np.uint32)), N
        inv = _dct(rt, 3, g[f"inv_in_{N}"].astype(np.float64), np.float64)
        assert np.array_equal(inv.view(np.uint64), g[f"inv_out_{N}"].view(np.uint64)), N


def test_large_bluestein_lengths_vs_oracle(rt):
    """Bluestein lengths 601..4096 (every 40th, and the largest) vs the oracle."""
    blue = [N for N in range(601, 4097) if rt.hb_rt_uses_bluestein(N)]
    rng = np.random.default_rng(11)
    for N in blue[::40] + [blue[-1]]:
        x = (rng.standard_normal((2, N)) * 60).astype(np.float32)
        a = _dct(rt, 2, x, np.float32)
        assert np.array_equal(a.view(np.uint32), O.dct_n(x, 2, np.float32).view(np.uint32)), N
        y = rng.integers(-3000, 3000, (2, N)).astype(np.float64)
        b = _dct(rt, 3, y, np.float64)
        assert np.array_equal(b.view(np.uint64), O.dct_n(y, 3, np.float64).view(np.uint64)), N
