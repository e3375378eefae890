"""Golden fixtures for the §8(f) row-4 plug-ins: YCrCb (src/YCrCb.py) and
LloydMax (src/LloydMax.py), run through the reference's own, unmodified glue
under /opt/conda/bin/python3.9 (numpy 1.26, tifffile 2021.7.2) with the
tests/golden/shims stand-ins (A12: color_transforms.YCrCb as OpenCV's integer
RGB<->YCrCb; A13: scalar_quantization.LloydMax_quantization as the textbook
Lloyd-Max design).  Build container only:

    python tests/golden/make_golden_plugins.py

What the fixtures pin is the glue: numpy.histogram of each channel, the +1,
the files (_params.txt, _centroids_<c>.gz), the dtype chain (float32 k ->
uint8 in 2D-DCT.py, uint8 k in LloydMax.py, int16 -> uint16 in YCrCb.py),
the offsets, TIFF bytes and decoded pixels.  The shims' arithmetic itself is
unpinned (neither package nor OpenCV is here).  Also recorded:
2D-DCT.py / 2D-DWT.py with -t YCrCb, run with the YCrCb shim raising if
called, equal the -t YCoCg runs byte for byte (both modules bind from_RGB /
to_RGB from color_transforms.YCoCg at import, 2D-DCT.py:22-23,
2D-DWT.py:19-20; -t only picks the base class, whose methods they override).
"""
import glob
import gzip
import io
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import PY39, REF_SRC, synth, tiff_pixels  # noqa: E402


def run(runner, module, sub, in_fn, out_fn, flags, extra_env=None):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(HERE, "shims") + os.pathsep + REF_SRC
    env["VCF_GOLDEN_HIDE_IMAGECODECS"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    env.update(extra_env or {})
    cmd = [PY39, "-W", "ignore", os.path.join(HERE, runner), module, sub, in_fn, out_fn] + flags
    r = subprocess.run(cmd, env=env, cwd=REF_SRC, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference run failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return int([l for l in r.stdout.splitlines() if l.startswith("RESULT_BYTES")][0].split()[1])


def side_files():
    """/tmp/encoded_params.txt and /tmp/encoded_centroids_<c>.gz (LloydMax.py:85-107)."""
    out = {}
    if os.path.exists("/tmp/encoded_params.txt"):
        out["params"] = np.frombuffer(open("/tmp/encoded_params.txt", "rb").read(), np.uint8)
    for fn in sorted(glob.glob("/tmp/encoded_centroids_*.gz")):
        c = int(fn.rsplit("_", 1)[1].split(".")[0])
        with gzip.GzipFile(fn, "r") as f:
            out[f"centroids_{c}"] = np.load(io.BytesIO(f.read()), allow_pickle=False)
    return out


def clear_side_files():
    for fn in glob.glob("/tmp/encoded_params.txt") + glob.glob("/tmp/encoded_centroids_*.gz"):
        os.remove(fn)


# name, kind, H, W, seed, module, runner, flags
CASES = [
    ("dct_lm_smooth_61x77", "smooth", 61, 77, 21, "2D-DCT", "_run_ref.py", ["-a", "LloydMax"]),
    ("dct_lm_rand_64x72_m2048_q16", "rand", 64, 72, 22, "2D-DCT", "_run_ref.py",
     ["-a", "LloydMax", "-m", "-2048", "-n", "2047", "-q", "16"]),
    ("dct_lm_smooth_57x63_x_m512", "smooth", 57, 63, 23, "2D-DCT", "_run_ref.py",
     ["-a", "LloydMax", "-x", "-m", "-512", "-n", "511", "-q", "8"]),
    ("dct_lm_smooth_64x64_p", "smooth", 64, 64, 24, "2D-DCT", "_run_ref.py",
     ["-a", "LloydMax", "-p", "-B", "8", "-m", "-1024", "-n", "1023"]),
    ("dct_lm_flat_48x56_b16", "flat", 48, 56, 25, "2D-DCT", "_run_ref.py",
     ["-a", "LloydMax", "-B", "16", "-m", "-2048", "-n", "2047", "-q", "64"]),
    ("lm_smooth_61x77", "smooth", 61, 77, 26, "LloydMax", "_run_ref_codec.py", []),
    ("lm_rand_40x48_q64", "rand", 40, 48, 27, "LloydMax", "_run_ref_codec.py", ["-q", "64"]),
    ("lm_extreme_32x40_q5_m16", "extreme", 32, 40, 28, "LloydMax", "_run_ref_codec.py",
     ["-q", "5", "-m", "16", "-n", "200"]),
    ("ycrcb_smooth_61x77", "smooth", 61, 77, 29, "YCrCb", "_run_ref_codec.py", ["-q", "32"]),
    ("ycrcb_rand_40x48_q5", "rand", 40, 48, 30, "YCrCb", "_run_ref_codec.py", ["-q", "5"]),
    ("ycrcb_extreme_32x40_q1", "extreme", 32, 40, 31, "YCrCb", "_run_ref_codec.py", ["-q", "1"]),
    ("ycrcb_lm_smooth_61x77", "smooth", 61, 77, 32, "YCrCb", "_run_ref_codec.py", ["-a", "LloydMax", "-q", "16"]),
]

# -t YCrCb on the transform codecs == -t YCoCg (the YCrCb shim raises if called)
SAME_CASES = [
    ("dct_t_ycrcb_smooth_61x77", "smooth", 61, 77, 33, "2D-DCT", ["-q", "7"]),
    ("dct_t_ycrcb_rand_40x48_x", "rand", 40, 48, 34, "2D-DCT", ["-x"]),
    ("dwt_t_ycrcb_smooth_64x72", "smooth", 64, 72, 35, "2D-DWT", ["-l", "3", "-w", "bior4.4"]),
]


def do_case(tmp, name, kind, H, W, seed, module, runner, flags):
    rgb = synth(kind, H, W, seed)
    in_fn = os.path.join(tmp, f"{name}.png")
    Image.fromarray(rgb).save(in_fn)
    enc = os.path.join(tmp, f"{name}_enc")
    dec = os.path.join(tmp, f"{name}_dec.png")
    clear_side_files()
    nbytes = run(runner, module, "encode", in_fn, enc, flags)
    side = side_files()
    tif = open(enc + ".tif", "rb").read()
    k = tiff_pixels(enc + ".tif")
    run(runner, module, "decode", enc, dec, flags)
    decoded = np.array(Image.open(dec))
    arrays = dict(rgb=rgb, k=k, decoded=decoded, tif=np.frombuffer(tif, np.uint8), **side)
    if os.path.exists(enc + "_shape.bin"):
        arrays["shape_bin"] = np.frombuffer(open(enc + "_shape.bin", "rb").read(), np.uint8)
    np.savez_compressed(os.path.join(HERE, f"plug_{name}.npz"), **arrays)
    clear_side_files()
    return dict(name=name, kind=kind, H=H, W=W, seed=seed, module=module, flags=flags,
                encode_bytes=nbytes, k_dtype=str(k.dtype), k_shape=list(k.shape),
                side_files=sorted(side))


def same_case(tmp, name, kind, H, W, seed, module, flags):
    """-t YCrCb vs -t YCoCg on the same input: every output file byte-equal."""
    rgb = synth(kind, H, W, seed)
    in_fn = os.path.join(tmp, f"{name}.png")
    Image.fromarray(rgb).save(in_fn)
    outs = {}
    for ct in ("YCoCg", "YCrCb"):
        d = os.path.join(tmp, f"{name}_{ct}")
        os.makedirs(d)
        enc, dec = os.path.join(d, "enc"), os.path.join(d, "dec.png")
        env = {"VCF_GOLDEN_YCRCB_UNUSED": "1"}
        run("_run_ref.py", module, "encode", in_fn, enc, flags + ["-t", ct], env)
        run("_run_ref.py", module, "decode", enc, dec, flags + ["-t", ct], env)
        files = {}
        for fn in sorted(os.listdir(d)):
            files[fn] = open(os.path.join(d, fn), "rb").read() if not fn.endswith(".png") \
                else np.array(Image.open(os.path.join(d, fn))).tobytes()
        outs[ct] = files
    assert outs["YCoCg"] == outs["YCrCb"], name
    return dict(name=name, module=module, flags=flags, files=sorted(outs["YCrCb"]), equal=True)


def make_hist():
    """numpy 1.26's histogram(x, bins=hi-lo+1, range=(lo, hi)) on float32 data at and
    around the bin edges, and on uint8 / int16 data (LloydMax.py:99-103)."""
    code = r"""
import sys, numpy as np
rng = np.random.Generator(np.random.PCG64(77))
out = {}
for i, (lo, hi) in enumerate([(0, 255), (-2048, 2047), (-512, 511), (16, 200), (-3, 3)]):
    n = hi - lo + 1
    e = np.linspace(lo, hi, n + 1, dtype=np.float32)
    near = np.concatenate([e, np.nextafter(e, np.float32(-np.inf)), np.nextafter(e, np.float32(np.inf))])
    x = np.concatenate([near, rng.uniform(lo - 5, hi + 5, 20000).astype(np.float32),
                        np.arange(lo - 2, hi + 3).astype(np.float32)]).astype(np.float32)
    out[f"f32_x_{i}"] = x
    out[f"f32_h_{i}"] = np.histogram(x, bins=n, range=(lo, hi))[0]
    xi = rng.integers(max(lo - 3, -32768), hi + 4, 5000).astype(np.int16)
    out[f"i16_x_{i}"] = xi
    out[f"i16_h_{i}"] = np.histogram(xi, bins=n, range=(lo, hi))[0]
    if lo >= 0:
        xu = rng.integers(0, 256, 5000).astype(np.uint8)
        out[f"u8_x_{i}"] = xu
        out[f"u8_h_{i}"] = np.histogram(xu, bins=n, range=(lo, hi))[0]
np.savez_compressed(sys.argv[1], **out)
"""
    subprocess.run([PY39, "-W", "ignore", "-c", code, os.path.join(HERE, "plug_histograms.npz")], check=True)


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    manifest = dict(generator="tests/golden/make_golden_plugins.py",
                    reference="src/YCrCb.py, src/LloydMax.py, src/2D-DCT.py, src/2D-DWT.py (unmodified glue)",
                    assumptions="A12 (color_transforms.YCrCb = OpenCV integer RGB<->YCrCb), "
                                "A13 (LloydMax_Quantizer, textbook Lloyd-Max): unpinned",
                    cases=[], same_as_ycocg=[])
    make_hist()
    with tempfile.TemporaryDirectory() as tmp:
        for c in CASES:
            manifest["cases"].append(do_case(tmp, *c))
            print("done", c[0], flush=True)
        for c in SAME_CASES:
            manifest["same_as_ycocg"].append(same_case(tmp, *c))
            print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_plugins.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
