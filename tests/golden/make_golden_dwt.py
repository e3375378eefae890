"""Golden fixtures for the 2D-DWT path, made by the reference itself.

Run in the build container (NOT on the GPU box):

    python tests/golden/make_golden_dwt.py

It drives the reference's unmodified src/2D-DWT.py encode_fn/decode_fn (with
YCoCg.py, deadzone.py, no_filter.py, TIFF.py, entropy_image_coding.py,
parser.py) under /opt/conda/bin/python3.9 -- pywt 1.1.1, tifffile 2021.7.2
-- with tests/golden/shims on PYTHONPATH for the un-vendored packages
(DWT2D.color_dyadic_DWT = assumption A6: per-channel pywt.wavedec2 /
waverec2, mode 'per').  Per case it stores the input frame, the pixels of
every subband file ({enc}_LL_{l}.tif u16, {enc}_{LH,HL,HH}_{r}.tif u8), the
bytes of the LL and finest-HH files, and the decoded frame.  dwt_pywt.npz
holds pywt.wavedec2/waverec2 on random float64 planes (transform-level pins).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import PY39, REF_SRC, synth  # noqa: E402

CASES = [
    # name, kind, H, W, seed, reference CLI flags (shared by encode/decode)
    ("smooth_64x64_bior_l3", "smooth", 64, 64, 20, ["-w", "bior4.4", "-l", "3"]),
    ("rand_64x72_db5_l2", "rand", 64, 72, 21, ["-l", "2"]),
    ("smooth_61x77_bior_l3", "smooth", 61, 77, 22, ["-w", "bior4.4", "-l", "3"]),
    ("rand_40x48_db5_l1_q7", "rand", 40, 48, 23, ["-l", "1", "-q", "7"]),
    ("smooth_160x256_bior_l5", "smooth", 160, 256, 24, ["-w", "bior4.4", "-l", "5"]),
    ("smooth_160x256_db5_l5_q16", "smooth", 160, 256, 25, ["-l", "5", "-q", "16"]),
    ("flat_48x56_bior_l2_q1", "flat", 48, 56, 26, ["-w", "bior4.4", "-l", "2", "-q", "1"]),
    ("extreme_32x40_db5_l2", "extreme", 32, 40, 27, ["-l", "2"]),
]


def run_ref(sub, in_fn, out_fn, flags):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(HERE, "shims") + os.pathsep + REF_SRC
    env["VCF_GOLDEN_HIDE_IMAGECODECS"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [PY39, "-W", "ignore", os.path.join(HERE, "_run_ref.py"), "2D-DWT", sub, in_fn, out_fn] + flags
    r = subprocess.run(cmd, env=env, cwd=REF_SRC, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference run failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return int([l for l in r.stdout.splitlines() if l.startswith("RESULT_BYTES")][0].split()[1])


def tiff_arrays(fns):
    code = ("import sys,numpy as np,tifffile;"
            "np.savez(sys.argv[1],**{str(i):tifffile.imread(f) for i,f in enumerate(sys.argv[2:])})")
    out = fns[0] + ".npz"
    subprocess.run([PY39, "-W", "ignore", "-c", code, out] + fns, check=True)
    d = np.load(out)
    return [d[str(i)] for i in range(len(fns))]


def levels_of(flags):
    return int(flags[flags.index("-l") + 1]) if "-l" in flags else 5


def do_case(tmp, name, kind, H, W, seed, flags):
    rgb = synth(kind, H, W, seed)
    in_fn = os.path.join(tmp, f"{name}.png")
    Image.fromarray(rgb).save(in_fn)
    enc = os.path.join(tmp, f"{name}_enc")
    dec = os.path.join(tmp, f"{name}_dec.png")
    nbytes = run_ref("encode", in_fn, enc, flags)
    L = levels_of(flags)
    names = [f"LL_{L}"] + [f"{s}_{r}" for r in range(L, 0, -1) for s in ("LH", "HL", "HH")]
    fns = [f"{enc}_{n}.tif" for n in names]
    arrays = dict(zip(names, tiff_arrays(fns)))
    run_ref("decode", enc, dec, flags)
    arrays["rgb"] = rgb
    arrays["decoded"] = np.array(Image.open(dec))
    arrays["tif_LL"] = np.frombuffer(open(fns[0], "rb").read(), np.uint8)
    arrays["tif_HH_1"] = np.frombuffer(open(f"{enc}_HH_1.tif", "rb").read(), np.uint8)
    np.savez_compressed(os.path.join(HERE, f"dwt_{name}.npz"), **arrays)
    return dict(name=name, kind=kind, H=H, W=W, seed=seed, flags=flags, levels=L, encode_bytes=nbytes,
                subbands=names, decoded_shape=list(arrays["decoded"].shape))


def make_pywt_vectors():
    code = r"""
import sys, numpy as np, pywt
rng = np.random.Generator(np.random.PCG64(4321))
out = {}
for wname in ('db5', 'bior4.4'):
    for (H, W, L) in ((37, 53, 3), (64, 64, 3), (160, 96, 4), (80, 120, 4)):
        x = rng.standard_normal((H, W)) * 100
        c = pywt.wavedec2(x, wname, mode='per', level=L)
        tag = f"{wname}_{H}x{W}_l{L}"
        out[f"fwd_in_{tag}"] = x
        out[f"fwd_{tag}_0"] = c[0]
        for l in range(1, L + 1):
            for s in range(3):
                out[f"fwd_{tag}_{l}_{s}"] = c[l][s]
        # inverse of integer-valued coefficients (what the decoder sees)
        ci = [np.rint(c[0] / 7).astype(np.int16) * 7] + \
             [tuple(np.rint(b / 5).astype(np.int16) * 5 for b in r) for r in c[1:]]
        y = pywt.waverec2(ci, wname, mode='per')
        out[f"inv_{tag}_0"] = ci[0]
        for l in range(1, L + 1):
            for s in range(3):
                out[f"inv_{tag}_{l}_{s}"] = ci[l][s]
        out[f"inv_out_{tag}"] = y
np.savez_compressed(sys.argv[1], **out)
"""
    subprocess.run([PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "dwt_pywt.npz")], check=True)


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    make_pywt_vectors()
    cases = []
    with tempfile.TemporaryDirectory() as tmp:
        for c in CASES:
            cases.append(do_case(tmp, *c))
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_dwt.json"), "w") as f:
        json.dump(dict(generator="tests/golden/make_golden_dwt.py",
                       reference="Sistemas-Multimedia/VCF src/2D-DWT.py encode_fn/decode_fn (unmodified glue)",
                       python="/opt/conda/bin/python3.9: pywt 1.1.1, tifffile 2021.7.2",
                       assumptions="tests/golden/shims (SURVEY.md Appendix A: A4, A5, A6, A9)",
                       cases=cases), f, indent=1)


if __name__ == "__main__":
    main()
