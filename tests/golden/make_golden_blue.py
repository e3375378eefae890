"""Golden fixtures for the block sizes pocketfft plans with Bluestein (fftblue
over a complex cfftp of length good_size_cmplx(2N - 1)).

Run in the build container (NOT on the GPU box):

    python tests/golden/make_golden_blue.py

1. cfft_blue.npz: scipy.fft.fft / ifft (pypocketfft c2c, the cfftp plan
   Bluestein runs on) under the reference's python3.9 / scipy 1.7.1, complex64
   and complex128, for the lengths the Bluestein plans of N <= 600 use (and
   small ones that exercise each pass): pins the cfftp restatement alone.
2. blocks_blue.npz: scipy.fftpack dct / idct (norm='ortho') for every length
   <= 600 that pocketfft_r plans with Bluestein, float32 forward on YCoCg-like
   inputs and float64 inverse on int16 inputs (assumptions A1/A2), as
   make_golden_radg.py does for the rfftp lengths.
3. dct_<case>.npz: the reference's own 2D-DCT.py encode_fn/decode_fn
   (unmodified glue, shims as in make_golden.py) at -B 191 and -B 478
   (= 2 x 239, a composite Bluestein length).
4. manifest_blue.json: lengths and cases.
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

B_CASES = [
    # name, kind, H, W, seed, flags
    ("b191_smooth_191x200", "smooth", 191, 200, 61, ["-B", "191"]),
    ("b478_smooth_240x250_q7", "smooth", 240, 250, 62, ["-B", "478", "-q", "7"]),
]


def good_size_cmplx(n):
    best = None
    f11 = 1
    while f11 < 2 * n + 64:
        f7 = f11
        while f7 < 2 * n + 64:
            f5 = f7
            while f5 < 2 * n + 64:
                f3 = f5
                while f3 < 2 * n + 64:
                    f2 = f3
                    while f2 < n:
                        f2 *= 2
                    if best is None or f2 < best:
                        best = f2
                    f3 *= 3
                f5 *= 5
            f7 *= 7
        f11 *= 11
    return best


def run39(code, out):
    subprocess.run([G.PY39, "-W", "ignore", "-c", code, out], check=True)


def main():
    if not os.path.exists(G.PY39) or not os.path.isdir(G.REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    from oracle import oracle as O
    blue = [n for n in range(1, 601) if not O.dct_supported(n)]
    cl = sorted(set([good_size_cmplx(2 * n - 1) for n in blue] +
                    [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 16, 20, 22, 24, 28, 32, 40, 44, 48, 56, 64, 72,
                     77, 80, 88, 96, 121, 128, 169, 176, 192]))
    run39(r"""
import sys, numpy as np, scipy.fft as F
rng = np.random.Generator(np.random.PCG64(4321))
out = {}
for N in %s:
    for dt, nm in ((np.complex64, 'c64'), (np.complex128, 'c128')):
        x = (rng.standard_normal((1, N)) + 1j * rng.standard_normal((1, N))).astype(dt)
        out[f'x_{nm}_{N}'] = x
        out[f'fwd_{nm}_{N}'] = F.fft(x, axis=-1)
        out[f'bwd_{nm}_{N}'] = F.ifft(x, axis=-1, norm='forward')
np.savez_compressed(sys.argv[1], **out)
""" % cl, os.path.join(HERE, "cfft_blue.npz"))
    run39(r"""
import sys, numpy as np
from scipy.fftpack import dct, idct
rng = np.random.Generator(np.random.PCG64(8766))
out = {}
for N in %s:
    fi = (rng.integers(-512, 509, (3, N)) / 4).astype(np.float32)
    out[f"fwd_in_{N}"] = fi
    out[f"fwd_out_{N}"] = dct(fi, norm='ortho', axis=-1)
    ii = (rng.integers(-40, 41, (3, N)) * rng.integers(1, 65, (3, 1))).astype(np.int16)
    out[f"inv_in_{N}"] = ii
    out[f"inv_out_{N}"] = idct(ii, norm='ortho', axis=-1)
np.savez_compressed(sys.argv[1], **out)
""" % blue, os.path.join(HERE, "blocks_blue.npz"))
    manifest = dict(generator="tests/golden/make_golden_blue.py",
                    reference="src/2D-DCT.py encode_fn/decode_fn (unmodified glue); scipy.fftpack dct/idct; "
                              "scipy.fft fft/ifft (pypocketfft c2c)",
                    python="/opt/conda/bin/python3.9: scipy 1.7.1, tifffile 2021.7.2",
                    bluestein_lengths=blue, cfft_lengths=cl, cases=[])
    with tempfile.TemporaryDirectory() as tmp:
        for c in B_CASES:
            manifest["cases"].append(G.do_case(tmp, *c))
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_blue.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
