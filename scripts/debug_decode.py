"""GPU debug: where does the decode kernel differ from the oracle?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import vcf_amd.dct as D
from oracle import oracle as O
from vcf_amd.device import set_device
set_device(0)
rng = np.random.Generator(np.random.PCG64(0))
for (H, W) in [(8, 8), (8, 16), (16, 8), (64, 72), (8, 2048), (64, 128)]:
    for Q in (32, 7):
        rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        k = O.encode_frame(rgb, Q)
        g = D.decode(k, H, W, Q)
        r = O.decode_frame(k, H, W, Q)
        bad = np.argwhere(g != r)
        print(H, W, Q, "mismatch", len(bad), "of", g.size)
        for b in bad[:6]:
            y, x, c = b
            print("   ", tuple(b), "gpu", g[y, x], "ref", r[y, x])
# constant index planes: isolate channels
for c in range(3):
    k = np.full((8, 8, 3), 128, np.uint8)
    k[0, 0, c] = 130
    g = D.decode(k, 8, 8, 32); r = O.decode_frame(k, 8, 8, 32)
    print("DC only ch", c, "gpu", g[0, :3].tolist(), "ref", r[0, :3].tolist(), "eq", np.array_equal(g, r))
