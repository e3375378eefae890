"""Golden block modes and GOP outputs of IPP_DCT.py's -R (rdo_lambda > 0) path,
made by the reference's own code.

    /opt/conda/bin/python3.9 tests/golden/make_golden_ipp_rdo.py

Runs under the reference's python3.9 (numpy 1.x, scipy 1.7.1 = pocketfft).
src/IPP_DCT.py imports av, cv2 and imageio at module level (absent here), so
the class IPP and the module functions it uses are extracted from its AST and
executed unmodified, with:
  * cv2.cvtColor(RGB2GRAY) restated by OpenCV's documented fixed-point
    formula (assumption A10, as make_golden_ipp.py);
  * scipy.fftpack's dct/idct (the module's own import, :17);
  * for temporal_filter's spatial codec, encode_decode_proxy (:595-626) is
    the 2D-DCT B=8 encode + decode of the C oracle (oracle/vcf_oracle.c, pinned
    to the reference's own 2D-DCT.py runs by tests/test_oracle.py), the same
    round trip the reference makes through lossless PNG temporaries.
Recorded:
  * blocks_*: for frame pairs (cur, comp) and several lambdas, the mode of
    every full block from IPP.rdo_block_decision on the luma blocks, the two
    get_rate values (inter, intra) and the returned distortion of the chosen
    mode;
  * seq_*: IPP.temporal_filter(frames, gop) with rdo_lambda > 0: each P
    frame's motion field and mode map, the frames handed to the spatial
    codec, and the reconstructed frames.
"""
import ast
import json
import os
import sys

import numpy as np
from scipy.fftpack import dct, idct

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src/IPP_DCT.py"
sys.path.insert(0, ROOT)


class _Cv2:
    COLOR_RGB2GRAY = 7

    @staticmethod
    def cvtColor(img, code):
        assert code == _Cv2.COLOR_RGB2GRAY
        r, g, b = (img[..., c].astype(np.int64) for c in range(3))
        return ((4899 * r + 9617 * g + 1868 * b + 8192) >> 14).astype(np.uint8)


class _Log:
    def __getattr__(self, name):
        return lambda *a, **k: None


def load():
    from concurrent.futures import ThreadPoolExecutor
    from typing import List, Tuple
    tree = ast.parse(open(REF).read())
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("_three_step_search", "_process_block_row")]
    ipp = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "IPP"]
    ns = {"np": np, "dct": dct, "idct": idct, "cv2": _Cv2, "logging": _Log(), "ThreadPoolExecutor": ThreadPoolExecutor,
          "List": List, "Tuple": Tuple}
    exec(compile(ast.Module(body=keep + ipp, type_ignores=[]), REF, "exec"), ns)
    return ns


class _Args:
    def __init__(self, qss):
        self.QSS = qss


class _Codec:
    """encode_decode_proxy over the oracle's 2D-DCT (B=8, deadzone Q)."""

    def __init__(self, qss):
        from oracle import oracle as O
        self.O = O
        self.args = _Args(qss)
        self.coded = []

    def encode_decode_proxy(self, img, frame_type, seq_idx):
        H, W = img.shape[:2]
        k = self.O.encode_frame(img, self.args.QSS, 0)
        self.coded.append((frame_type, img.copy()))
        return self.O.decode_frame(k, H, W, self.args.QSS, 0), int(k.nbytes)


def frames_seq(H, W, n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    y, x = np.mgrid[0:H + 40, 0:W + 40].astype(np.float64)
    base = np.stack([128 + 60 * np.sin(x / 13 + c) + 50 * np.cos(y / 11 - c) for c in range(3)], -1)
    base += rng.normal(0, 6, base.shape)
    out = []
    for t in range(n):
        dy, dx = 3 * t % 17, (2 * t + (t * t) % 5) % 19
        f = base[20 + dy - 8:20 + dy - 8 + H, 20 + dx - 8:20 + dx - 8 + W].copy()
        if t % 3 == 2:   # an occluding patch appears: blocks the prediction cannot follow
            f[H // 4:H // 2, W // 3:W // 2] = rng.integers(0, 256, (H // 2 - H // 4, W // 2 - W // 3, 3))
        out.append(np.clip(np.rint(f), 0, 255).astype(np.uint8))
    return out


def comp_mix(cur, bs, seed):
    """A compensation that predicts some blocks well, some badly."""
    rng = np.random.Generator(np.random.PCG64(seed))
    comp = cur.astype(np.int32).copy()
    H, W = cur.shape[:2]
    for by in range(H // bs):
        for bx in range(W // bs):
            sl = (slice(by * bs, (by + 1) * bs), slice(bx * bs, (bx + 1) * bs))
            kind = (by * 7 + bx * 3 + seed) % 4
            if kind == 0:
                comp[sl] += rng.integers(-3, 4, comp[sl].shape)
            elif kind == 1:
                comp[sl] += rng.integers(-25, 26, comp[sl].shape)
            elif kind == 2:
                comp[sl] = rng.integers(0, 256, comp[sl].shape)
            else:
                comp[sl] = np.roll(comp[sl], 3, axis=1) + 10
    return np.clip(comp, 0, 255).astype(np.uint8)


def block_modes(ns, cur, comp, bs, qss, lam):
    ipp = ns["IPP"](None, bs, 8, False, 0, rdo_lambda=lam)
    rates = []
    orig = ipp.get_rate

    def rec_rate(data, is_intra=False):
        r = orig(data, is_intra)
        rates.append(r)
        return r

    ipp.get_rate = rec_rate
    H, W = cur.shape[:2]
    modes = np.zeros((H // bs, W // bs), np.uint8)
    dist = np.zeros((H // bs, W // bs))
    rr = np.zeros((H // bs, W // bs, 2))
    for i in range(0, H - bs + 1, bs):
        for j in range(0, W - bs + 1, bs):
            cg = _Cv2.cvtColor(cur[i:i + bs, j:j + bs], _Cv2.COLOR_RGB2GRAY)
            pg = _Cv2.cvtColor(comp[i:i + bs, j:j + bs], _Cv2.COLOR_RGB2GRAY)
            rates.clear()
            mode, _, d = ipp.rdo_block_decision(cg, pg, qss)
            modes[i // bs, j // bs] = 1 if mode == "I" else 0
            dist[i // bs, j // bs] = d
            rr[i // bs, j // bs] = rates
    return modes, dist, rr


def main():
    ns = load()
    np.random.seed(0)   # rdo_block_decision draws np.random.rand() for its debug print
    arrays, cases = {}, []
    for name, H, W, bs, qss in (("blocks_64x96_bs16", 64, 96, 16, 32), ("blocks_72x120_bs8", 72, 120, 8, 32),
                                ("blocks_48x64_bs16_q7", 48, 64, 16, 7)):
        cur = frames_seq(H, W, 1, len(cases) + 11)[0]
        comp = comp_mix(cur, bs, len(cases))
        arrays[f"{name}_cur"], arrays[f"{name}_comp"] = cur, comp
        lams = (0.01, 0.5, 3.0, 50.0)
        for li, lam in enumerate(lams):
            m, d, r = block_modes(ns, cur, comp, bs, qss, lam)
            arrays[f"{name}_l{li}_modes"], arrays[f"{name}_l{li}_dist"], arrays[f"{name}_l{li}_rates"] = m, d, r
            print(name, lam, "I-blocks", int(m.sum()), "of", m.size, flush=True)
        cases.append(dict(name=name, H=H, W=W, bs=bs, qss=qss, lambdas=list(lams)))
    seqs = []
    for name, H, W, n, gop, bs, sr, qss, lam in (("seq_64x96_bs16", 64, 96, 6, 4, 16, 8, 32, 0.5),
                                                 ("seq_72x120_bs8", 72, 120, 4, 4, 8, 8, 32, 3.0)):
        frames = frames_seq(H, W, n, 100 + len(seqs))
        codec = _Codec(qss)
        ipp = ns["IPP"](codec, bs, sr, False, 0, rdo_lambda=lam)
        I_infos, P_infos, mv_infos, recon = ipp.temporal_filter(frames, gop)
        arrays[f"{name}_frames"] = np.stack(frames)
        arrays[f"{name}_mv"] = np.stack([m["mv"] for m in mv_infos])
        arrays[f"{name}_modes"] = np.stack([m["modes"] for m in mv_infos])
        arrays[f"{name}_coded"] = np.stack([img for _, img in codec.coded])
        arrays[f"{name}_recon"] = np.stack(recon)
        seqs.append(dict(name=name, H=H, W=W, n=n, gop=gop, bs=bs, sr=sr, qss=qss, rdo_lambda=lam,
                         coded_types=[t for t, _ in codec.coded],
                         I_blocks=[int(m["modes"].sum()) for m in mv_infos]))
        print(name, seqs[-1]["I_blocks"], flush=True)
    np.savez_compressed(os.path.join(HERE, "ipp_rdo.npz"), **arrays)
    json.dump(dict(generator="tests/golden/make_golden_ipp_rdo.py (python3.9, scipy 1.7.1)",
                   reference="Sistemas-Multimedia/VCF src/IPP_DCT.py class IPP (rdo_block_decision, get_rate, "
                             "temporal_filter with rdo_lambda > 0), AST-extracted and executed unmodified",
                   assumptions="A10: cv2 RGB2GRAY = (4899R + 9617G + 1868B + 8192) >> 14; spatial codec = "
                               "2D-DCT B=8 via the pinned C oracle",
                   block_cases=cases, seq_cases=seqs), open(os.path.join(HERE, "manifest_ipp_rdo.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
