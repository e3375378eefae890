"""Golden code-streams of CBAHC (src/CBAHC.py), made by the reference itself.

    python tests/golden/make_golden_cbahc.py

Imports the reference's src/CBAHC.py unmodified under /opt/conda/bin/python3.9
(bitarray present; tests/golden/shims stand in for cv2 and the un-vendored
packages the import chain pulls in) and calls CoDec.compress_fn /
decompress_fn on small uint8 arrays (the reference's Python coder rebuilds a
Huffman tree per symbol, so the streams are short).  Stores the symbols, the
.huf bytes and the side file's content (shape, order, nbits).
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import PY39, REF_SRC  # noqa: E402

RUNNER = r"""
import sys, os, io, gzip, pickle, argparse, numpy as np, warnings
warnings.filterwarnings('ignore')
sys.argv = ['CBAHC.py', 'encode']
import importlib
m = importlib.import_module('CBAHC')
spec = np.load(os.environ['CBAHC_IN'])
out = {}
for name in spec.files:
    img = spec[name]
    order = int(name.split('_o')[1])
    tmp = os.environ['CBAHC_TMP'] + '/' + name
    args = argparse.Namespace(subparser_name='encode', order=order, debug=False)
    c = m.CoDec(args)
    b = c.compress_fn(img, tmp).getvalue()
    with gzip.open(tmp + '_adaptive_huffman_tree.pkl.gz', 'rb') as f:
        shape = np.load(f)
        meta = pickle.load(f)
    dec = m.CoDec(argparse.Namespace(subparser_name='decode', order=order, debug=False)).decompress_fn(b, tmp)
    assert np.array_equal(dec, img)
    out[name + '_huf'] = np.frombuffer(b, np.uint8)
    out[name + '_nbits'] = np.array([meta['nbits']])
    out[name + '_shape'] = np.asarray(shape)
np.savez_compressed(os.environ['CBAHC_OUT'], **out)
"""


def main():
    if not os.path.exists(PY39) or not os.path.isdir(REF_SRC):
        sys.exit("needs /opt/conda/bin/python3.9 and /root/reference (build container only)")
    rng = np.random.Generator(np.random.PCG64(55))
    inputs = {
        "laplace_o0": np.clip(np.rint(rng.laplace(128, 3, (20, 30, 3))), 0, 255).astype(np.uint8),
        "laplace_o1": np.clip(np.rint(rng.laplace(128, 3, (16, 25, 3))), 0, 255).astype(np.uint8),
        "laplace_o2": np.clip(np.rint(rng.laplace(128, 2, (12, 20, 3))), 0, 255).astype(np.uint8),
        "uniform_o0": rng.integers(0, 256, (40, 40), dtype=np.uint8),
        "const_o0": np.full((10, 33), 200, np.uint8),
        "runs_o1": np.repeat(rng.integers(0, 256, 60, dtype=np.uint8), 20).reshape(30, 40),
    }
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        inp = os.path.join(tmp, "in.npz")
        np.savez(inp, **inputs)
        out = os.path.join(tmp, "out.npz")
        env = dict(os.environ, PYTHONPATH=os.path.join(HERE, "shims") + os.pathsep + REF_SRC,
                   CBAHC_IN=inp, CBAHC_OUT=out, CBAHC_TMP=tmp, VCF_GOLDEN_HIDE_IMAGECODECS="1")
        r = subprocess.run([PY39, "-W", "ignore", "-c", RUNNER], env=env, cwd=REF_SRC, capture_output=True,
                           text=True)
        if r.returncode != 0:
            sys.exit(r.stdout[-3000:] + r.stderr[-3000:])
        res = dict(np.load(out))
    arrays = {}
    for k, v in inputs.items():
        arrays[f"{k}_sym"] = v
        for suffix in ("huf", "nbits", "shape"):
            arrays[f"{k}_{suffix}"] = res[f"{k}_{suffix}"]
    np.savez_compressed(os.path.join(HERE, "cbahc.npz"), **arrays)
    json.dump(dict(generator="tests/golden/make_golden_cbahc.py",
                   reference="Sistemas-Multimedia/VCF src/CBAHC.py CoDec.compress_fn/decompress_fn (unmodified)",
                   python="/opt/conda/bin/python3.9 (bitarray)",
                   cases=[dict(name=k, order=int(k.split("_o")[1]), shape=list(v.shape),
                               nbits=int(res[f"{k}_nbits"][0])) for k, v in inputs.items()]),
              open(os.path.join(HERE, "manifest_cbahc.json"), "w"), indent=1)
    print("ok", {k: int(res[f"{k}_nbits"][0]) for k in inputs})


if __name__ == "__main__":
    main()
