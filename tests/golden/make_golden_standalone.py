"""Golden fixtures for the reference's stand-alone codecs (SURVEY.md §8(b)'s
CLI surface): src/YCoCg.py, src/deadzone.py, src/TIFF.py, src/CBAAC.py
(--order 0/1) and src/CBAHC.py (--order 0/1), each run as its own program
(tests/golden/_run_ref_main.py: runpy with __name__ == "__main__", the
reference's unmodified files) under /opt/conda/bin/python3.9 (numpy 1.26,
tifffile 2021.7.2, bitarray) with the tests/golden/shims stand-ins for the
un-vendored packages: A4 (color_transforms.YCoCg), A5 (deadzone quantizer),
A8 (arithmetic_coding: the CBAAC coder's bytes are pinned only as far as A8
is), cv2.  Build container only:

    python tests/golden/make_golden_standalone.py

Each fixture holds the input image, the encoded file's bytes, the side file
where there is one (CBAHC's /tmp/encoded_adaptive_huffman_tree.pkl.gz is
recorded as its decompressed numpy/pickle payload fields: shape, order,
nbits), the decoded image and, for the lossy codecs, the index array.
"""
import gzip
import io
import json
import os
import pickle
import shutil
import subprocess
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import PY39, REF_SRC, synth, tiff_pixels  # noqa: E402

EXT = {"YCoCg": ".tif", "deadzone": ".tif", "TIFF": ".tif", "CBAAC": ".adpt_arith", "CBAHC": ".huf"}
SIDE = "/tmp/encoded_adaptive_huffman_tree.pkl.gz"


# name, kind, H, W, seed, module, flags
CASES = [
    ("ycocg_smooth_61x77", "smooth", 61, 77, 41, "YCoCg", []),
    ("ycocg_rand_40x48_q5", "rand", 40, 48, 42, "YCoCg", ["-q", "5"]),
    ("ycocg_extreme_32x40_q1", "extreme", 32, 40, 43, "YCoCg", ["-q", "1"]),
    ("ycocg_flat_48x56_q64", "flat", 48, 56, 44, "YCoCg", ["-q", "64"]),
    ("ycocg_lm_smooth_61x77", "smooth", 61, 77, 45, "YCoCg", ["-a", "LloydMax", "-q", "16"]),
    ("deadzone_smooth_61x77", "smooth", 61, 77, 46, "deadzone", []),
    ("deadzone_rand_40x48_q7", "rand", 40, 48, 47, "deadzone", ["-q", "7"]),
    ("deadzone_extreme_32x40_q1", "extreme", 32, 40, 48, "deadzone", ["-q", "1"]),
    ("deadzone_rand_33x35_q255", "rand", 33, 35, 49, "deadzone", ["-q", "255"]),
    ("tiff_smooth_61x77", "smooth", 61, 77, 50, "TIFF", []),
    ("tiff_rand_300x300", "rand", 300, 300, 51, "TIFF", []),
    ("cbaac_smooth_24x20_o0", "smooth", 24, 20, 52, "CBAAC", []),
    ("cbaac_smooth_24x20_o1", "smooth", 24, 20, 53, "CBAAC", ["--order", "1"]),
    ("cbaac_rand_16x18_o2", "rand", 16, 18, 54, "CBAAC", ["--order", "2"]),
    ("cbahc_smooth_24x20_o0", "smooth", 24, 20, 55, "CBAHC", []),
    ("cbahc_smooth_24x20_o1", "smooth", 24, 20, 56, "CBAHC", ["--order", "1"]),
]


def clear():
    for fn in ["/tmp/original.png", "/tmp/decoded.png", SIDE, "/tmp/encoded_params.txt"] + \
              [f"/tmp/encoded{e}" for e in set(EXT.values())] + [f"/tmp/encoded_centroids_{c}.gz" for c in range(3)]:
        if os.path.exists(fn):
            os.remove(fn)


def do_case(name, kind, H, W, seed, module, flags):
    rgb = synth(kind, H, W, seed)
    clear()
    Image.fromarray(rgb).save("/tmp/original.png")
    # the options follow the subcommand (the reference's subparsers own them)
    cmd_flags = flags
    _run(module, ["encode"] + cmd_flags)
    enc = f"/tmp/encoded{EXT[module]}"
    arrays = dict(rgb=rgb, enc=np.frombuffer(open(enc, "rb").read(), np.uint8))
    if EXT[module] == ".tif":
        shutil.copy(enc, "/tmp/_golden.tif")
        arrays["k"] = tiff_pixels("/tmp/_golden.tif")
    side = {}
    if module == "CBAHC":
        with gzip.open(SIDE, "rb") as f:
            arrays["side_shape"] = np.load(f, allow_pickle=False)
            meta = pickle.load(f)   # our own generator's file, written by the reference just now
        arrays["side_order"] = np.array(meta["order"])
        arrays["side_nbits"] = np.array(meta["nbits"])
        side = dict(order=int(meta["order"]), nbits=int(meta["nbits"]))
    if os.path.exists("/tmp/encoded_params.txt"):
        arrays["params"] = np.frombuffer(open("/tmp/encoded_params.txt", "rb").read(), np.uint8)
    _run(module, ["decode"] + cmd_flags)
    arrays["decoded"] = np.array(Image.open("/tmp/decoded.png"))
    np.savez_compressed(os.path.join(HERE, f"sa_{name}.npz"), **arrays)
    clear()
    return dict(name=name, kind=kind, H=H, W=W, seed=seed, module=module, flags=flags,
                enc_bytes=int(arrays["enc"].size), decoded_dtype=str(arrays["decoded"].dtype), **side)


def _run(module, argv):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.join(HERE, "shims") + os.pathsep + REF_SRC
    env["VCF_GOLDEN_HIDE_IMAGECODECS"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    cmd = [PY39, "-W", "ignore", os.path.join(HERE, "_run_ref_main.py"), module] + argv
    r = subprocess.run(cmd, env=env, cwd=REF_SRC, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference run failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    manifest = dict(generator="tests/golden/make_golden_standalone.py",
                    reference="src/YCoCg.py, src/deadzone.py, src/TIFF.py, src/CBAAC.py, src/CBAHC.py "
                              "(unmodified, run as programs)",
                    assumptions="A4 (YCoCg), A5 (deadzone), A8 (CBAAC coder bytes), A13 (LloydMax design)",
                    cases=[])
    for c in CASES:
        manifest["cases"].append(do_case(*c))
        print("done", c[0], flush=True)
    with open(os.path.join(HERE, "manifest_standalone.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
