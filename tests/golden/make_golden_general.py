"""Golden fixtures for block sizes other than 8 and for the -L search.

Run in the build container (NOT on the GPU box):

    python tests/golden/make_golden_general.py

1. blocks_general.npz: scipy.fftpack dct/idct (norm='ortho') of random
   vectors for every length the restatement covers, under the reference's
   python3.9 / scipy 1.7.1 (pocketfft): float32 forward on YCoCg-like
   inputs, float64 inverse on int16 inputs (assumptions A1/A2).
2. dct_b<B>_<case>.npz: the reference's own 2D-DCT.py encode_fn/decode_fn
   (unmodified glue, shims for the un-vendored packages as in make_golden.py)
   run with -B <B>: input frame, the .tif's indices and bytes, _shape.bin,
   decoded frame.
3. dct_L_<case>.npz: 2D-DCT.py encode with -L <lambda>: the block size
   optimize_block_size (:533-579) picks, its per-size J values from the
   reference's debug log (:576), and the encode_fn output at that size.
   optimize_block_size reads the hard-coded /tmp/original.png
   (entropy_image_coding.py:67), so the frame is written there first.
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402

LENGTHS = [1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 15, 16, 18, 20, 24, 25, 27, 30, 32, 36, 40, 45, 48, 50, 54, 60, 64,
           72, 75, 80, 81, 90, 96, 100, 108, 120, 125, 128]   # the 5-smooth N <= 128

B_CASES = [
    # name, kind, H, W, seed, flags
    ("b4_rand_64x72", "rand", 64, 72, 20, ["-B", "4"]),
    ("b16_smooth_61x77", "smooth", 61, 77, 21, ["-B", "16"]),
    ("b32_rand_40x48_x", "rand", 40, 48, 22, ["-B", "32", "-x"]),
    ("b2_smooth_33x35_q7", "smooth", 33, 35, 23, ["-B", "2", "-q", "7"]),
    ("b64_smooth_64x128_q1", "smooth", 64, 128, 24, ["-B", "64", "-q", "1"]),
    ("b128_flat_128x128", "flat", 128, 128, 25, ["-B", "128"]),
    ("b12_rand_50x50_q5", "rand", 50, 50, 26, ["-B", "12", "-q", "5"]),
    ("b3_rand_30x20", "rand", 30, 20, 27, ["-B", "3"]),
    ("b1_rand_5x7", "rand", 5, 7, 28, ["-B", "1", "-q", "3"]),
    ("b96_smooth_96x96_x", "smooth", 96, 96, 29, ["-B", "96", "-x"]),
    ("b5_rand_37x41", "rand", 37, 41, 30, ["-B", "5"]),
    ("b10_smooth_64x70_q7", "smooth", 64, 70, 31, ["-B", "10", "-q", "7"]),
    ("b15_rand_45x46_x", "rand", 45, 46, 32, ["-B", "15", "-x"]),
    ("b20_smooth_83x61", "smooth", 83, 61, 33, ["-B", "20"]),
    ("b25_flat_75x50_q1", "flat", 75, 50, 34, ["-B", "25", "-q", "1"]),
    ("b45_smooth_90x101", "smooth", 90, 101, 35, ["-B", "45"]),
    ("b100_rand_100x120_q5", "rand", 100, 120, 36, ["-B", "100", "-q", "5"]),
    ("b125_smooth_130x125", "smooth", 130, 125, 37, ["-B", "125"]),
    ("b27_rand_54x60", "rand", 54, 60, 38, ["-B", "27"]),
    ("b81_smooth_81x90_x", "smooth", 81, 90, 39, ["-B", "81", "-x"]),
]
L_CASES = [
    # name, kind, H, W, seed, lambda, extra flags
    ("L_smooth_128x256_l1000", "smooth", 128, 256, 40, "1000", []),
    ("L_rand_128x128_l10", "rand", 128, 128, 41, "10", []),
    ("L_smooth_256x128_l1e5_q7", "smooth", 256, 128, 42, "100000", ["-q", "7"]),
]


def make_blocks():
    code = r"""
import sys, numpy as np
from scipy.fftpack import dct, idct
rng = np.random.Generator(np.random.PCG64(4321))
out = {}
for N in %s:
    fi = (rng.integers(-512, 509, (64, N)) / 4).astype(np.float32)
    out[f"fwd_in_{N}"] = fi
    out[f"fwd_out_{N}"] = dct(fi, norm='ortho', axis=-1)
    ii = (rng.integers(-40, 41, (64, N)) * rng.integers(1, 65, (64, 1))).astype(np.int16)
    out[f"inv_in_{N}"] = ii
    out[f"inv_out_{N}"] = idct(ii, norm='ortho', axis=-1)
np.savez_compressed(sys.argv[1], **out)
""" % LENGTHS
    subprocess.run([G.PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "blocks_general.npz")], check=True)


def run_ref_log(sub, in_fn, out_fn, flags):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(HERE, "shims") + os.pathsep + G.REF_SRC
    env["VCF_GOLDEN_HIDE_IMAGECODECS"] = "1"
    env["VCF_GOLDEN_LOG"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [G.PY39, "-W", "ignore", os.path.join(HERE, "_run_ref.py"), "2D-DCT", sub, in_fn, out_fn] + flags
    r = subprocess.run(cmd, env=env, cwd=G.REF_SRC, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference run failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stdout


def do_L_case(tmp, name, kind, H, W, seed, lam, flags):
    rgb = G.synth(kind, H, W, seed)
    orig = "/tmp/original.png"   # hard-coded in optimize_block_size -> encode_read()
    backup = None
    if os.path.exists(orig):
        backup = os.path.join(tmp, "original_backup.png")
        shutil.copy(orig, backup)
    try:
        Image.fromarray(rgb).save(orig)
        enc = os.path.join(tmp, f"{name}_enc")
        out = run_ref_log("encode", orig, enc, ["-L", lam] + flags)
    finally:
        if backup:
            shutil.copy(backup, orig)
        else:
            os.remove(orig)
    js = [(int(m.group(2)), float(m.group(1))) for m in re.finditer(r"J=(\S+) for block_size=(\d+)", out)]
    bs = int(re.search(r"RESULT_BLOCK_SIZE (\d+)", out).group(1))
    k = G.tiff_pixels(enc + ".tif")
    tif = open(enc + ".tif", "rb").read()
    np.savez_compressed(os.path.join(HERE, f"dct_{name}.npz"), rgb=rgb, k=k, tif=np.frombuffer(tif, np.uint8),
                        J_block_sizes=np.array([b for b, _ in js]), J=np.array([j for _, j in js]),
                        block_size=np.array(bs))
    return dict(name=name, kind=kind, H=H, W=W, seed=seed, flags=["-L", lam] + flags, chosen_block_size=bs,
                J=dict((str(b), j) for b, j in js))


def main():
    if not os.path.exists(G.PY39) or not os.path.isdir(G.REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    manifest = dict(generator="tests/golden/make_golden_general.py",
                    reference="src/2D-DCT.py encode_fn/decode_fn and optimize_block_size (unmodified glue)",
                    python="/opt/conda/bin/python3.9: scipy 1.7.1, tifffile 2021.7.2",
                    lengths=LENGTHS, cases=[], L_cases=[])
    make_blocks()
    with tempfile.TemporaryDirectory() as tmp:
        for c in B_CASES:
            manifest["cases"].append(G.do_case(tmp, *c))
            print("done", c[0], flush=True)
        for c in L_CASES:
            manifest["L_cases"].append(do_L_case(tmp, *c))
            print("done", c[0], manifest["L_cases"][-1]["chosen_block_size"], flush=True)
    with open(os.path.join(HERE, "manifest_general.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
