"""Golden traces of the CBAAC context model, made by the reference's own code.

    python tests/golden/make_golden_cbaac.py

src/CBAAC.py cannot be imported here (its module body needs bitarray, cv2 and
the un-vendored arithmetic_coding package), so the two classes the coder is
driven by -- AdaptiveModel (:17-47) and ContextManager (:49-69) -- are
extracted from the file's AST and executed as they are.  For synthetic
symbol streams the script replays CBAAC.CoDec._encode's model loop (:114-131:
history deque of `order` zeros, get_model(tuple(history)), get_range, update,
append) and records the (low, high, total) triple handed to the arithmetic
coder for every symbol.  Those triples are everything the model contributes
to the code-stream; the coder itself (arithmetic_coding, not vendored) is
assumption A8.
"""
import ast
import json
import os
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/CBAAC.py"


def load_classes():
    tree = ast.parse(open(REF).read())
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in ("AdaptiveModel", "ContextManager")]
    ns = {}
    exec(compile(ast.Module(body=keep, type_ignores=[]), REF, "exec"), ns)
    return ns["AdaptiveModel"], ns["ContextManager"]


def trace(symbols, order, ContextManager):
    ctx = ContextManager(order=order)
    history = deque([0] * order, maxlen=order if order > 0 else 1)
    out = np.empty((len(symbols), 3), np.int64)
    for i, s in enumerate(symbols):
        key = tuple(history) if order > 0 else ()
        m = ctx.get_model(key)
        out[i] = m.get_range(int(s))
        m.update(int(s))
        if order > 0:
            history.append(int(s))
    return out


def streams():
    rng = np.random.Generator(np.random.PCG64(77))
    laplace = np.clip(np.rint(rng.laplace(128, 3, 60000)), 0, 255).astype(np.uint8)   # k+128 indices
    uniform = rng.integers(0, 256, 30000, dtype=np.uint8)
    runs = np.repeat(rng.integers(0, 256, 400, dtype=np.uint8), 50)                    # 20000, long runs
    skewed = np.where(rng.random(40000) < 0.97, 128, rng.integers(0, 256, 40000)).astype(np.uint8)
    return dict(laplace=laplace, uniform=uniform, runs=runs, skewed=skewed)


def main():
    _, ContextManager = load_classes()
    arrays, cases = {}, []
    for name, sym in streams().items():
        for order in (0, 1, 2):
            if order == 2 and name in ("uniform",):
                continue
            t = trace(sym, order, ContextManager)
            arrays[f"sym_{name}"] = sym
            arrays[f"trace_{name}_o{order}"] = t.astype(np.int32)
            cases.append(dict(stream=name, order=order, n=int(len(sym)),
                              rescales=int(np.sum(np.diff(t[:, 2]) < 0))))
    np.savez_compressed(os.path.join(HERE, "cbaac_model.npz"), **arrays)
    json.dump(dict(generator="tests/golden/make_golden_cbaac.py",
                   reference="Sistemas-Multimedia/VCF src/CBAAC.py AdaptiveModel/ContextManager (AST-extracted, "
                             "executed unmodified)",
                   cases=cases), open(os.path.join(HERE, "manifest_cbaac.json"), "w"), indent=1)
    print(cases)


if __name__ == "__main__" and len(__import__("sys").argv) == 1:
    main()


# ---- tiled CBAAC (the GPU entropy stage) ----------------------------
# The tiled variant splits the flattened symbol stream into consecutive
# segments of seg_len symbols and runs CBAAC.CoDec._encode's model loop
# (:114-131) on each segment from scratch: a fresh ContextManager, history
# reset to `order` zeros.  These traces are the reference's own classes run
# exactly that way, segment by segment.
#
#     python tests/golden/make_golden_cbaac.py tiled

TILED_SEG = 24576   # a multiple of 256 (the GPU kernel's chunk); long enough for order-0 rescales


def main_tiled():
    _, ContextManager = load_classes()
    arrays, cases = {}, []
    s = streams()
    for name in ("laplace", "skewed"):
        sym = s[name]
        arrays[f"sym_{name}"] = sym
        for order in (0, 1):
            parts = [trace(sym[i:i + TILED_SEG], order, ContextManager) for i in range(0, len(sym), TILED_SEG)]
            arrays[f"trace_{name}_o{order}"] = np.concatenate(parts).astype(np.int32)
            cases.append(dict(stream=name, order=order, n=int(len(sym)), seg_len=TILED_SEG, segments=len(parts)))
    np.savez_compressed(os.path.join(HERE, "cbaac_tiled.npz"), **arrays)
    json.dump(dict(generator="tests/golden/make_golden_cbaac.py tiled",
                   reference="Sistemas-Multimedia/VCF src/CBAAC.py AdaptiveModel/ContextManager (AST-extracted, "
                             "executed unmodified), one fresh ContextManager per segment",
                   cases=cases), open(os.path.join(HERE, "manifest_cbaac_tiled.json"), "w"), indent=1)
    print(cases)


if __name__ == "__main__" and len(__import__("sys").argv) > 1 and __import__("sys").argv[1] == "tiled":
    main_tiled()
