"""The C-ABI library without a GPU: it builds, loads, and exports exactly what
include/*.h declares; argument validation runs on the host and reports the
reference's errors (2D-DCT.py:199-200 raises ValueError for ndim != 3).
No compute entry point is called with real buffers here."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

from conftest import ROOT

import vcf_amd._lib as L


def _declared(header="vcf_amd.h"):
    names = []
    for h in glob.glob(os.path.join(ROOT, "include", header)):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s]*?[\s*](vcf_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_library_builds_and_loads():
    lib = L.lib()
    assert os.path.exists(L.lib_path())
    major, minor = ctypes.c_int(), ctypes.c_int()
    assert lib.vcf_version(ctypes.byref(major), ctypes.byref(minor)) == 0
    assert major.value >= 0 and minor.value >= 0


def test_every_declared_symbol_is_exported():
    lib = L.lib()
    names = _declared()
    assert len(names) >= 25, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    """Every declared entry point has argtypes in vcf_amd/_lib.py, and no extra."""
    declared = set(_declared()) - {"vcf_last_error"}
    assert declared == set(L.SIGNATURES), (declared ^ set(L.SIGNATURES))


def test_ab_library_is_separate():
    """The A/B kernel variants (include/vcf_amd_ab.h) live in libvcf_amd_ab.so
    only: the product library does not export them, the A/B library does."""
    ab = _declared("vcf_amd_ab.h")
    assert set(ab) == set(L.AB_SIGNATURES), set(ab) ^ set(L.AB_SIGNATURES)
    assert not set(ab) & set(_declared())
    lib, abl = L.lib(), L.ab()
    assert not [n for n in ab if hasattr(lib, n)]
    assert not [n for n in ab if not hasattr(abl, n)]


def test_padded_shape_is_host_only():
    Hp, Wp = ctypes.c_int32(), ctypes.c_int32()
    lib = L.lib()
    assert lib.vcf_dct_padded_shape(61, 77, 8, ctypes.byref(Hp), ctypes.byref(Wp)) == 0
    assert (Hp.value, Wp.value) == (64, 80)
    assert lib.vcf_dct_padded_shape(0, 77, 8, ctypes.byref(Hp), ctypes.byref(Wp)) == L.VCF_ERR_INVALID


@pytest.mark.parametrize("args,status", [
    (dict(H=0), L.VCF_ERR_INVALID),              # not an image
    (dict(block_size=5000), L.VCF_ERR_UNSUPPORTED),  # beyond the run-time path's 4096
    (dict(block_size=5000, flags=2), L.VCF_ERR_UNSUPPORTED),
    (dict(Q=0), L.VCF_ERR_INVALID),
    (dict(flags=8), L.VCF_ERR_INVALID),
    (dict(n_frames=-1), L.VCF_ERR_INVALID),
])
def test_argument_errors_before_any_device_work(args, status):
    """check_args() rejects bad calls before touching HIP (null device
    pointers would otherwise fault)."""
    a = dict(n_frames=1, H=8, W=8, block_size=8, Q=32, flags=0)
    a.update(args)
    dummy = ctypes.c_void_p(16)   # never dereferenced: validation fails first
    rc = L.lib().vcf_dct_dz_encode(dummy, a["n_frames"], a["H"], a["W"], a["block_size"], a["Q"],
                                   a["flags"], dummy, None)
    assert rc == status
    assert L.lib().vcf_last_error()  # a message is recorded


def test_null_buffers_rejected():
    rc = L.lib().vcf_dct_dz_decode(None, 1, 8, 8, 8, 32, 0, None, None)
    assert rc == L.VCF_ERR_INVALID


def test_status_mapping():
    with pytest.raises(ValueError):
        L.check(L.VCF_ERR_INVALID)
    with pytest.raises(NotImplementedError):
        L.check(L.VCF_ERR_UNSUPPORTED)
    with pytest.raises(RuntimeError):
        L.check(L.VCF_ERR_HIP)


def test_product_never_imports_the_oracle():
    """vcf_amd/ has no path to oracle/ (no CPU fallback)."""
    for p in glob.glob(os.path.join(ROOT, "vcf_amd", "**", "*.py"), recursive=True):
        src = open(p).read()
        assert "oracle" not in re.sub(r"#.*|\"\"\".*?\"\"\"", "", src, flags=re.S), p


def test_block_size_coverage():
    """-B sizes with a HIP transform: every B up to 4096 -- compiled kernels
    for the 5-smooth B <= 128, the run-time path for the rest, rfftp plans and
    the lengths pocketfft plans with Bluestein (tests/golden/manifest_blue.json)."""
    lib = L.lib()
    have = [b for b in range(0, 601) if lib.vcf_dct_block_size_supported(b)]
    assert have == list(range(1, 601))
    assert lib.vcf_dct_block_size_supported(4096) and not lib.vcf_dct_block_size_supported(4097)


def test_perceptual_tables_match_the_oracle():
    """-p's resized JPEG tables (host only): B = 8 is the reference's own
    table, integer area scales average, and every B the oracle's
    restatement of cv2.resize gives (unpinned for B != 8: no cv2 here)."""
    from oracle import oracle as O
    lib = L.lib()
    for B in list(range(1, 33)) + [49, 64, 100, 128, 130, 200]:
        y = np.empty((B, B), np.uint8)
        c = np.empty((B, B), np.uint8)
        assert lib.vcf_dct_perceptual_tables(B, y.ctypes.data, c.ctypes.data) == 0
        yo, co = O.perceptual_tables(B)
        assert np.array_equal(y, yo) and np.array_equal(c, co), B
    y8, c8 = O.perceptual_tables(8)
    assert y8[0].tolist() == [16, 11, 10, 16, 24, 40, 51, 61] and c8[0].tolist() == [17, 18, 24, 47, 99, 99, 99, 99]
    y4, _ = O.perceptual_tables(4)
    assert y4[0, 0] == 13   # (16 + 11 + 12 + 12) / 4 = 12.75, rounded
    assert lib.vcf_dct_perceptual_tables(0, y.ctypes.data, c.ctypes.data) == L.VCF_ERR_INVALID


def test_product_path_fails_loudly_without_the_library(tmp_path):
    """No CPU fallback: with the HIP library absent, the codec raises instead of computing."""
    import subprocess
    import sys
    code = ("import numpy as np, vcf_amd.dct as D\n"
            "try:\n    D.encode(np.zeros((8, 8, 3), np.uint8), 32)\n"
            "except ImportError as e:\n    print('raised', e)\n")
    env = dict(os.environ, VCF_AMD_LIB=str(tmp_path / "absent.so"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert p.returncode == 0, p.stderr[-1500:]
    assert p.stdout.startswith("raised") and "no CPU fallback" in p.stdout
