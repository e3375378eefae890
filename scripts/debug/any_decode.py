import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import vcf_amd.dct as D
from oracle import oracle as O
for B in (16, 32, 12, 24):
    for (H, W) in ((37, 47), (32, 32), (48, 48), (2 * B + 5, 3 * B - 1), (64, 64), (16, 48)):
        rgb = np.random.default_rng(1).integers(0, 256, (H, W, 3), np.uint8)
        k = D.encode(rgb, 32, 0, block_size=B)
        a = D.decode(k, H, W, 32, 0, block_size=B)
        b = O.decode_frame_b(k, H, W, B, 32, 0)
        bad = np.argwhere((a != b).any(-1))
        k32 = D.encode_k32(rgb, 32, 0, block_size=B)
        a32 = D.decode_k32(k32, H, W, 32, 0, block_size=B)
        b32 = O.decode_frame_b(k32, H, W, B, 32, 0)
        bad32 = np.argwhere((a32 != b32).any(-1))
        print(B, H, W, "bad", len(bad), bad[:1].tolist(), bad[-1:].tolist(), "k32 bad", len(bad32), flush=True)
