"""Golden fixtures for block sizes with a prime factor above 5 (pocketfft's
generic radfg/radbg passes) and for the lengths pocketfft plans with Bluestein.

Run in the build container (NOT on the GPU box):

    python tests/golden/make_golden_radg.py

1. blocks_radg.npz: scipy.fftpack dct/idct (norm='ortho') under the
   reference's python3.9 / scipy 1.7.1 (pocketfft) for every length 1..200
   whose factorisation has a prime above 5, float32 forward on YCoCg-like
   inputs and float64 inverse on int16 inputs (assumptions A1/A2), as
   make_golden_general.py does for the 5-smooth lengths.
2. dct_<case>.npz: the reference's own 2D-DCT.py encode_fn/decode_fn
   (unmodified glue, shims as in make_golden.py) run with -B 7, 11, 13, 14,
   21, 49, 98, 130 and 200 (padding, -x, several -q).
3. manifest_radg.json: the lengths, the cases, and the lengths <= 600 the
   restatement plans with Bluestein (pocketfft_r's cost model), for which the
   HIP path returns VCF_ERR_UNSUPPORTED.
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import make_golden as G  # noqa: E402


def smooth5(n):
    for p in (2, 3, 5):
        while n % p == 0:
            n //= p
    return n == 1


B_CASES = [
    # name, kind, H, W, seed, flags
    ("b7_rand_35x42", "rand", 35, 42, 50, ["-B", "7"]),
    ("b11_smooth_61x77", "smooth", 61, 77, 51, ["-B", "11"]),
    ("b13_rand_40x48_x", "rand", 40, 48, 52, ["-B", "13", "-x"]),
    ("b14_smooth_56x70_q7", "smooth", 56, 70, 53, ["-B", "14", "-q", "7"]),
    ("b21_flat_42x63_q1", "flat", 42, 63, 54, ["-B", "21", "-q", "1"]),
    ("b49_smooth_98x100", "smooth", 98, 100, 55, ["-B", "49"]),
    ("b98_rand_98x98_q5", "rand", 98, 98, 56, ["-B", "98", "-q", "5"]),
    ("b130_smooth_130x140_x", "smooth", 130, 140, 57, ["-B", "130", "-x"]),
    ("b200_smooth_200x210", "smooth", 200, 210, 58, ["-B", "200"]),
]


def make_blocks(lengths):
    code = r"""
import sys, numpy as np
from scipy.fftpack import dct, idct
rng = np.random.Generator(np.random.PCG64(8765))
out = {}
for N in %s:
    fi = (rng.integers(-512, 509, (4, N)) / 4).astype(np.float32)
    out[f"fwd_in_{N}"] = fi
    out[f"fwd_out_{N}"] = dct(fi, norm='ortho', axis=-1)
    ii = (rng.integers(-40, 41, (4, N)) * rng.integers(1, 65, (4, 1))).astype(np.int16)
    out[f"inv_in_{N}"] = ii
    out[f"inv_out_{N}"] = idct(ii, norm='ortho', axis=-1)
np.savez_compressed(sys.argv[1], **out)
""" % lengths
    subprocess.run([G.PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "blocks_radg.npz")], check=True)


def main():
    if not os.path.exists(G.PY39) or not os.path.isdir(G.REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    from oracle import oracle as O
    blue = [n for n in range(1, 601) if not O.dct_supported(n)]
    lengths = [n for n in range(1, 201) if not smooth5(n) and n not in blue]
    manifest = dict(generator="tests/golden/make_golden_radg.py",
                    reference="src/2D-DCT.py encode_fn/decode_fn (unmodified glue); scipy.fftpack dct/idct",
                    python="/opt/conda/bin/python3.9: scipy 1.7.1, tifffile 2021.7.2",
                    lengths=lengths, bluestein_lengths=blue, cases=[])
    make_blocks(lengths)
    with tempfile.TemporaryDirectory() as tmp:
        for c in B_CASES:
            manifest["cases"].append(G.do_case(tmp, *c))
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_radg.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
