"""The reference's stand-alone codecs on the GPU, through libvcf_amd.so and
the new CLIs (vcf_amd/cli/{YCoCg,deadzone,TIFF,CBAAC,CBAHC}.py): every file
and decoded image equals what the reference itself wrote
(tests/golden/sa_*.npz, make_golden_standalone.py: src/YCoCg.py,
deadzone.py, TIFF.py, CBAAC.py --order, CBAHC.py --order run as programs),
and the fused YCoCg/deadzone kernels equal the oracle on seeded sweeps."""
import os
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

from oracle import plugins as O
from test_standalone import cases, load, qss

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXT = {"YCoCg": ".tif", "deadzone": ".tif", "TIFF": ".tif", "CBAAC": ".adpt_arith", "CBAHC": ".huf"}


def _cli(module, sub, flags):
    r = subprocess.run([sys.executable, f"vcf_amd/cli/{module}.py", sub] + flags, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("c", cases(), ids=lambda c: c["name"])
def test_cli_reproduces_reference(c):
    """`python <module>.py encode|decode [flags]` with the reference's hard-wired
    /tmp/original.png -> /tmp/encoded<ext> -> /tmp/decoded.png."""
    z = load(c)
    for fn in ("/tmp/decoded.png", f"/tmp/encoded{EXT[c['module']]}"):
        if os.path.exists(fn):
            os.remove(fn)
    Image.fromarray(z["rgb"]).save("/tmp/original.png")
    _cli(c["module"], "encode", c["flags"])
    assert open(f"/tmp/encoded{EXT[c['module']]}", "rb").read() == z["enc"].tobytes()
    if "params" in z.files:
        assert open("/tmp/encoded_params.txt", "rb").read() == z["params"].tobytes()
    _cli(c["module"], "decode", c["flags"])
    assert np.array_equal(np.array(Image.open("/tmp/decoded.png")), z["decoded"])


@pytest.mark.parametrize("c", cases(("YCoCg", "deadzone")), ids=lambda c: c["name"])
def test_kernels_equal_reference_indices(c):
    from vcf_amd import plugins as PL
    if "LloydMax" in c["flags"]:
        pytest.skip("LloydMax path: covered by the CLI test")
    z = load(c)
    Q = qss(c)
    if c["module"] == "YCoCg":
        assert np.array_equal(PL.ycocg_dz_encode(z["rgb"], Q), z["k"])
        assert np.array_equal(PL.ycocg_dz_decode(z["k"], Q), z["decoded"])
    else:
        assert np.array_equal(PL.dz_u8_encode(z["rgb"], Q), z["k"])
        assert np.array_equal(PL.dz_u8_decode(z["k"], Q), z["decoded"])


@pytest.mark.parametrize("shape", [(1, 1), (1, 3), (7, 5), (33, 129), (64, 1023), (1080, 1920)])
@pytest.mark.parametrize("Q", [1, 3, 32, 255, 4096])
def test_kernels_equal_oracle(shape, Q):
    """Seeded sweeps: ragged pixel counts (4-pixel groups with tails), unaligned
    views, every Q class, random u16 indices for the decoders (wrapping)."""
    from vcf_amd import plugins as PL
    rng = np.random.Generator(np.random.PCG64(hash((shape, Q)) & 0xffff))
    rgb = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    assert np.array_equal(PL.ycocg_dz_encode(rgb, Q), O.ycocg_dz_encode(rgb, Q))
    k = rng.integers(0, 65536, shape + (3,), dtype=np.uint16)
    assert np.array_equal(PL.ycocg_dz_decode(k, Q), O.ycocg_dz_decode(k, Q))
    assert np.array_equal(PL.dz_u8_encode(rgb, Q), O.dz_u8_encode(rgb, Q))
    if Q <= 255:
        k8 = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
        assert np.array_equal(PL.dz_u8_decode(k8, Q), O.dz_u8_decode(k8, Q))
    # an odd byte offset: the kernels' unaligned paths
    big = rng.integers(0, 256, rgb.size + 1, dtype=np.uint8)
    v = big[1:].reshape(rgb.shape)
    assert np.array_equal(PL.dz_u8_encode(v, Q), O.dz_u8_encode(v, Q))


def test_unsupported_q():
    from vcf_amd import plugins as PL
    k = np.zeros((2, 2, 3), np.uint8)
    with pytest.raises(NotImplementedError):
        PL.dz_u8_decode(k, 256)
    with pytest.raises(NotImplementedError):
        PL.ycocg_dz_decode(k.astype(np.uint16), 40000)
    with pytest.raises(ValueError):
        PL.ycocg_dz_encode(np.zeros((2, 2, 3), np.uint8), 0)
