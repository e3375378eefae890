import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvcf_amd.so)")


def _manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_cases():
    return _manifest()["cases"]


def case_params(case):
    """(Q, flags) from the reference CLI flags recorded for a golden case."""
    fl = case["flags"]
    Q = int(fl[fl.index("-q") + 1]) if "-q" in fl else 32
    flags = (1 if "-x" in fl else 0) | (2 if "-p" in fl else 0)
    return Q, flags


def load_case(case):
    return np.load(os.path.join(GOLDEN, f"dct_{case['name']}.npz"))


@pytest.fixture(scope="session")
def manifest():
    return _manifest()
