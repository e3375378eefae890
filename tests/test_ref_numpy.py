"""bench.py's cpu_baseline legs (oracle/ref_numpy.py) against the reference's outputs.

The numpy restatement of 2D-DCT.py encode_fn is what `cpu_baseline` times
as "the reference's CPU path"; here it is pinned to the fixtures the
reference's unmodified glue produced (tests/golden/make_golden.py): every
committed case without -p, and the 512x512 cases of config C1 by SHA-256.
The vectorised form must equal the per-block loop bit for bit.
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

from conftest import GOLDEN, case_params, golden_cases, load_case
from oracle import ref_numpy as R


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _synth():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.synth


@pytest.mark.parametrize("case", [c for c in golden_cases() if "-p" not in c["flags"]], ids=lambda c: c["name"])
def test_ref_numpy_vs_reference(case):
    d = load_case(case)
    Q, flags = case_params(case)
    sub = not (flags & 1)
    assert np.array_equal(R.encode_frame_loop(d["rgb"], Q, sub), d["k"])
    assert np.array_equal(R.encode_frame(d["rgb"], Q, sub, workers=2), d["k"])


@pytest.mark.parametrize("name", ["smooth_512x512", "rand_512x512"])
def test_ref_numpy_c1_by_hash(manifest, name):
    case = [c for c in manifest["big_cases"] if c["name"] == name][0]
    rgb = _synth()(case["kind"], case["H"], case["W"], case["seed"])
    assert _sha(R.encode_frame(rgb, 32, workers=4)) == case["sha256"]["k"]
    assert _sha(R.encode_frame_loop(rgb[:64], 32)) == _sha(R.encode_frame(rgb[:64], 32))


def test_ref_numpy_matches_c_port_on_a_4k_strip():
    from vcf_amd.synthetic import synth_frame
    from oracle import oracle as O
    f = synth_frame(2160, 3840, 0)
    k = R.encode_frame(f, 32, workers=4)
    assert np.array_equal(k, O.encode_frame(f, 32))
    assert np.array_equal(R.encode_frame_loop(f[:16], 32), R.encode_frame(f[:16], 32))


def test_ref_numpy_rejects_non_rgb():
    with pytest.raises(ValueError):
        R.encode_frame(np.zeros((8, 8), np.uint8))
