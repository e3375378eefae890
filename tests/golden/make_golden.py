"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run in the build container (NOT on the GPU box, where neither the reference
nor python3.9 exists):

    python tests/golden/make_golden.py

It drives the reference's own glue (src/2D-DCT.py encode_fn/decode_fn with
src/YCoCg.py, src/deadzone.py, src/no_filter.py, src/TIFF.py,
src/entropy_image_coding.py, src/parser.py), unmodified, under
/opt/conda/bin/python3.9 (scipy 1.7.1 = pocketfft, tifffile 2021.7.2,
skimage 0.18.3), with tests/golden/shims on PYTHONPATH standing in for the
un-vendored upstream packages (assumptions A1-A9).

Outputs (all small): dct_<case>.npz holding the input frame, the quantization
indices the reference's TIFF carries, the .tif bytes (stdlib-zlib tifffile
path and, for one case, the imagecodecs/libdeflate path), the _shape.bin
bytes and the decoded frame; blocks.npz with scipy.fftpack 8x8 transforms;
manifest.json with the options of every case and SHA-256 digests of the
large (512x512, 1080p) cases whose arrays are not committed.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
PY39 = "/opt/conda/bin/python3.9"


def synth(kind, H, W, seed):
    """Synthetic inputs of SURVEY.md §8(d): S-rand, S-smooth, S-flat."""
    rng = np.random.Generator(np.random.PCG64(seed))
    if kind == "rand":
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if kind == "smooth":
        y, x = np.mgrid[0:H, 0:W].astype(np.float64)
        ch = []
        for c in range(3):
            v = 128 + 60 * np.sin(x / 97 + c) + 50 * np.cos(y / 61 - c) + rng.normal(0, 4, (H, W))
            ch.append(v)
        return np.clip(np.rint(np.stack(ch, -1)), 0, 255).astype(np.uint8)
    if kind == "flat":
        blocks = rng.integers(0, 256, ((H + 7) // 8, (W + 7) // 8, 3), dtype=np.uint8)
        return np.repeat(np.repeat(blocks, 8, 0), 8, 1)[:H, :W].copy()
    if kind == "extreme":
        v = rng.integers(0, 2, (H, W, 3), dtype=np.uint8) * 255
        return v
    raise ValueError(kind)


CASES = [
    # name, kind, H, W, seed, reference CLI flags (shared by encode/decode)
    ("rand_64x72", "rand", 64, 72, 0, []),
    ("smooth_61x77", "smooth", 61, 77, 1, []),
    ("flat_48x56", "flat", 48, 56, 2, []),
    ("extreme_32x40_q1", "extreme", 32, 40, 3, ["-q", "1"]),
    ("smooth_64x64_q1", "smooth", 64, 64, 4, ["-q", "1"]),
    ("smooth_64x64_q7", "smooth", 64, 64, 5, ["-q", "7"]),
    ("rand_64x64_q64", "rand", 64, 64, 6, ["-q", "64"]),
    ("rand_40x48_x", "rand", 40, 48, 7, ["-x"]),
    ("smooth_57x63_x_q5", "smooth", 57, 63, 8, ["-x", "-q", "5"]),
    ("smooth_64x64_p", "smooth", 64, 64, 9, ["-p"]),
    ("rand_48x64_p_q7", "rand", 48, 64, 10, ["-p", "-q", "7"]),
    ("flat_33x35_p_x", "flat", 33, 35, 11, ["-p", "-x"]),
    ("rand_8x8", "rand", 8, 8, 12, []),
    ("rand_1x1", "rand", 1, 1, 13, []),
    ("rand_3x17_q3", "rand", 3, 17, 14, ["-q", "3"]),
]
BIG_CASES = [
    ("smooth_512x512", "smooth", 512, 512, 100, []),   # config C1
    ("rand_512x512", "rand", 512, 512, 101, []),
]


def run_ref(sub, in_fn, out_fn, flags, hide_imagecodecs=True):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(HERE, "shims") + os.pathsep + REF_SRC
    env["VCF_GOLDEN_HIDE_IMAGECODECS"] = "1" if hide_imagecodecs else "0"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [PY39, "-W", "ignore", os.path.join(HERE, "_run_ref.py"), "2D-DCT", sub,
           in_fn, out_fn] + flags
    r = subprocess.run(cmd, env=env, cwd=REF_SRC, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference run failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return int([l for l in r.stdout.splitlines() if l.startswith("RESULT_BYTES")][0].split()[1])


def tiff_pixels(tif_fn):
    code = ("import sys,numpy as np,tifffile;a=tifffile.imread(sys.argv[1]);"
            "np.save(sys.argv[2],a)")
    out = tif_fn + ".npy"
    subprocess.run([PY39, "-W", "ignore", "-c", code, tif_fn, out], check=True)
    return np.load(out)


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def do_case(tmp, name, kind, H, W, seed, flags, store_arrays=True):
    rgb = synth(kind, H, W, seed)
    in_fn = os.path.join(tmp, f"{name}.png")
    Image.fromarray(rgb).save(in_fn)
    enc = os.path.join(tmp, f"{name}_enc")
    dec = os.path.join(tmp, f"{name}_dec.png")
    nbytes = run_ref("encode", in_fn, enc, flags)
    tif = open(enc + ".tif", "rb").read()
    shape_bin = open(enc + "_shape.bin", "rb").read()
    k = tiff_pixels(enc + ".tif")
    run_ref("decode", enc, dec, flags)
    decoded = np.array(Image.open(dec))
    meta = dict(name=name, kind=kind, H=H, W=W, seed=seed, flags=flags,
                encode_bytes=nbytes, k_shape=list(k.shape),
                sha256=dict(rgb=sha(rgb.tobytes()), k=sha(k.tobytes()), tif=sha(tif),
                            decoded=sha(decoded.tobytes())))
    if store_arrays:
        arrays = dict(rgb=rgb, k=k, decoded=decoded,
                      tif=np.frombuffer(tif, np.uint8), shape_bin=np.frombuffer(shape_bin, np.uint8))
        if name == "rand_64x72":
            # the same encode with imagecodecs importable: tifffile then uses libdeflate
            enc2 = os.path.join(tmp, f"{name}_enc_libdeflate")
            run_ref("encode", in_fn, enc2, flags, hide_imagecodecs=False)
            arrays["tif_libdeflate"] = np.frombuffer(open(enc2 + ".tif", "rb").read(), np.uint8)
        np.savez_compressed(os.path.join(HERE, f"dct_{name}.npz"), **arrays)
    return meta


def make_blocks():
    """scipy.fftpack 8x8 transforms under python3.9 (scipy 1.7.1)."""
    code = r"""
import sys, numpy as np
from scipy.fftpack import dct, idct
rng = np.random.Generator(np.random.PCG64(1234))
# YCoCg-domain inputs: multiples of 1/4 in [-128, 127]
fwd_in = (rng.integers(-512, 509, (2048, 8, 8)) / 4).astype(np.float32)
const = (np.arange(-512, 509) / 4).astype(np.float32)
fwd_in = np.concatenate([fwd_in, np.broadcast_to(const[:, None, None], (const.size, 8, 8))])
f = lambda b: dct(dct(b.T, norm='ortho').T, norm='ortho')
fwd_out = np.stack([f(b) for b in fwd_in])
inv_in = (rng.integers(-40, 41, (2048, 8, 8)) * rng.integers(1, 65, (2048, 1, 1))).astype(np.int16)
g = lambda b: idct(idct(b.T, norm='ortho').T, norm='ortho')
inv_out = np.stack([g(b) for b in inv_in])
np.savez_compressed(sys.argv[1], fwd_in=fwd_in, fwd_out=fwd_out, inv_in=inv_in, inv_out=inv_out)
"""
    subprocess.run([PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "blocks.npz")],
                   check=True)


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    manifest = dict(
        generator="tests/golden/make_golden.py",
        reference="Sistemas-Multimedia/VCF src/2D-DCT.py encode_fn/decode_fn (unmodified glue)",
        python="/opt/conda/bin/python3.9: scipy 1.7.1, tifffile 2021.7.2, skimage 0.18.3",
        assumptions="tests/golden/shims (SURVEY.md Appendix A: A1-A5, A7, A9)",
        tiff_path="tifffile stdlib-zlib path (imagecodecs hidden); tif_libdeflate = imagecodecs path",
        cases=[], big_cases=[])
    make_blocks()
    with tempfile.TemporaryDirectory() as tmp:
        for c in CASES:
            manifest["cases"].append(do_case(tmp, *c))
            print("done", c[0], flush=True)
        for c in BIG_CASES:
            manifest["big_cases"].append(do_case(tmp, *c, store_arrays=False))
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
