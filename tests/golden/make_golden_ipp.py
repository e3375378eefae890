"""Golden motion fields / compensation of IPP_DCT.py, made by the reference's code.

    python tests/golden/make_golden_ipp.py

src/IPP_DCT.py imports av, cv2 and imageio at module level, none of which
exist here, so the functions the IPP hot path runs are extracted from its AST
and executed as written: _three_step_search (:159-204), _process_block_row
(:207-246, full search and --fast) and IPP.motion_compensate (:378-395).
IPP.block_matching (:344-376) only adds cv2.cvtColor(RGB2GRAY); that is
restated with OpenCV's documented fixed-point formula for 8-bit images,
Y = (4899 R + 9617 G + 1868 B + 8192) >> 14 (assumption A10, SURVEY.md
§8(c): cv2 is not installed, so this is unpinned).
"""
import ast
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/IPP_DCT.py"


def load():
    tree = ast.parse(open(REF).read())
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("_three_step_search", "_process_block_row")]
    ipp = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "IPP"][0]
    mc = [n for n in ipp.body if isinstance(n, ast.FunctionDef) and n.name == "motion_compensate"][0]
    ns = {"np": np}
    exec(compile(ast.Module(body=keep + [mc], type_ignores=[]), REF, "exec"), ns)
    return ns


def gray(rgb):
    r, g, b = (rgb[..., c].astype(np.int64) for c in range(3))
    return ((4899 * r + 9617 * g + 1868 * b + 8192) >> 14).astype(np.uint8)


def block_matching(ns, ref, cur, bs, sr, fast):
    """IPP.block_matching (:344-376) with the rows run in order."""
    h, w = ref.shape[:2]
    rg, cg = gray(ref), gray(cur)
    mv = np.zeros((h // bs, w // bs, 2), np.float32)
    for i in range(0, h - bs + 1, bs):
        _, row = ns["_process_block_row"]((rg, cg, i, bs, sr, w, fast))
        for c, m in enumerate(row):
            mv[i // bs, c] = m
    return mv


def sequence(H, W, n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    y, x = np.mgrid[0:H + 40, 0:W + 40].astype(np.float64)
    base = np.stack([128 + 60 * np.sin(x / 13 + c) + 50 * np.cos(y / 11 - c) for c in range(3)], -1)
    base += rng.normal(0, 6, base.shape)
    frames = []
    for t in range(n):
        dy, dx = 3 * t % 17, (2 * t + (t * t) % 5) % 19     # varied motion, within +-8 of the previous frame
        f = base[20 + dy - 8:20 + dy - 8 + H, 20 + dx - 8:20 + dx - 8 + W]
        frames.append(np.clip(np.rint(f), 0, 255).astype(np.uint8))
    return frames


class _Self:
    def __init__(self, bs):
        self.block_size = bs


def main():
    ns = load()
    arrays, cases = {}, []
    for name, H, W, n, bs, sr in (("seq_64x96", 64, 96, 4, 16, 8), ("seq_72x120_bs8", 72, 120, 3, 8, 8),
                                  ("seq_50x70", 50, 70, 3, 16, 6)):
        frames = sequence(H, W, n, len(cases) + 3)
        arrays[f"{name}_frames"] = np.stack(frames)
        for fast in (False, True):
            mvs, comps = [], []
            for t in range(1, n):
                mv = block_matching(ns, frames[t - 1], frames[t], bs, sr, fast)
                comp = ns["motion_compensate"](_Self(bs), frames[t - 1], mv)
                mvs.append(mv)
                comps.append(comp)
            tag = f"{name}_{'fast' if fast else 'full'}"
            arrays[f"{tag}_mv"] = np.stack(mvs)
            arrays[f"{tag}_comp"] = np.stack(comps)
        cases.append(dict(name=name, H=H, W=W, n=n, bs=bs, sr=sr))
    np.savez_compressed(os.path.join(HERE, "ipp.npz"), **arrays)
    json.dump(dict(generator="tests/golden/make_golden_ipp.py",
                   reference="Sistemas-Multimedia/VCF src/IPP_DCT.py _process_block_row/_three_step_search/"
                             "IPP.motion_compensate (AST-extracted, executed unmodified)",
                   assumptions="A10: cv2 RGB2GRAY = (4899R + 9617G + 1868B + 8192) >> 14",
                   cases=cases), open(os.path.join(HERE, "manifest_ipp.json"), "w"), indent=1)
    print(cases)


if __name__ == "__main__":
    main()
