"""Golden fixtures for pywt's short-input branch of the inverse DWT (a subband
line shorter than half the filter: the coefficients wrap around more than
once), made by the reference and pywt 1.1.1 themselves.  Build container only:

    python tests/golden/make_golden_dwt_short.py

* dwt_short_pywt.npz: pywt.idwt(cA, cD, w, mode='periodization') and
  pywt.dwt(x, w, mode='periodization') on random float64 lines of every
  length 1 .. F/2 + 3 for every discrete wavelet pywt knows (the order of the
  products is what is pinned: outputs are compared bit for bit).
* dwt_short_<case>.npz + manifest_dwt_short.json: the unmodified
  src/2D-DWT.py encode_fn/decode_fn (make_golden_dwt.py's harness) on frames
  small enough that the last levels' subbands are shorter than F/2.
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden_dwt as G  # noqa: E402
from make_golden import PY39, REF_SRC  # noqa: E402

CASES = [
    ("short_20x24_db5_l5", "smooth", 20, 24, 40, ["-l", "5"]),
    ("short_13x17_bior_l4", "rand", 13, 17, 41, ["-w", "bior4.4", "-l", "4"]),
    ("short_33x35_db5_l4_q7", "smooth", 33, 35, 42, ["-l", "4", "-q", "7"]),
    ("short_9x40_sym8_l3", "rand", 9, 40, 43, ["-w", "sym8", "-l", "3"]),
    ("short_8x8_db10_l2", "extreme", 8, 8, 44, ["-w", "db10", "-l", "2"]),
    ("short_64x3_coif2_l2_q3", "smooth", 64, 3, 45, ["-w", "coif2", "-l", "2", "-q", "3"]),
]


def make_vectors():
    code = r"""
import sys, numpy as np, pywt
rng = np.random.Generator(np.random.PCG64(9876))
out = {}
names = pywt.wavelist(kind='discrete')
out['names'] = np.array(names)
for w in names:
    W = pywt.Wavelet(w); F2 = W.rec_len // 2
    for N in range(1, F2 + 4):
        a = rng.standard_normal(N) * 100; d = rng.standard_normal(N) * 100
        out[f'inv_a_{w}_{N}'] = a; out[f'inv_d_{w}_{N}'] = d
        out[f'inv_{w}_{N}'] = pywt.idwt(a, d, w, mode='periodization')
        x = rng.standard_normal(2 * N - (N & 1)) * 100
        cA, cD = pywt.dwt(x, w, mode='periodization')
        out[f'fwd_x_{w}_{N}'] = x; out[f'fwd_a_{w}_{N}'] = cA; out[f'fwd_d_{w}_{N}'] = cD
np.savez_compressed(sys.argv[1], **out)
"""
    subprocess.run([PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "dwt_short_pywt.npz")], check=True)


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    make_vectors()
    cases = []
    with tempfile.TemporaryDirectory() as tmp:
        for c in CASES:
            meta = G.do_case(tmp, *c)
            os.replace(os.path.join(HERE, f"dwt_{c[0]}.npz"), os.path.join(HERE, f"dwt_short_{c[0][6:]}.npz"))
            meta["file"] = f"dwt_short_{c[0][6:]}.npz"
            cases.append(meta)
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_dwt_short.json"), "w") as f:
        json.dump(dict(generator="tests/golden/make_golden_dwt_short.py",
                       reference="src/2D-DWT.py encode_fn/decode_fn (unmodified glue), pywt 1.1.1",
                       cases=cases), f, indent=1)


if __name__ == "__main__":
    main()
