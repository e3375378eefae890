"""Run the default DCT+deadzone decode of 64 4K frames N times (for rocprofv3
--pmc passes).  python scripts/dct_dec_once.py [N]; DENSE=1: uniform-random
frames (every coefficient nonzero: the decode's worst case), else S-smooth."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import vcf_amd.dct as D
from vcf_amd.device import DeviceBuffer, Stream, set_device
from vcf_amd.synthetic import synth_frame

set_device(0)
H, W, F, Q = 2160, 3840, 64, 32
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
Hp, Wp = D.padded_shape(H, W)
if os.environ.get("DENSE", "0") == "1":
    frames = [np.random.Generator(np.random.PCG64(s)).integers(0, 256, (H, W, 3), dtype=np.uint8) for s in range(4)]
else:
    frames = [synth_frame(H, W, s) for s in range(4)]
din = DeviceBuffer(F * H * W * 3)
for f in range(F):
    din.upload(frames[f % 4], offset=f * H * W * 3)
s = Stream()
dk = DeviceBuffer(F * Hp * Wp * 3)
D.encode_device(din, F, H, W, Q, out=dk, stream=s)
dout = DeviceBuffer(F * H * W * 3)
for _ in range(n):
    D.decode_device(dk, F, H, W, Q, out=dout, stream=s)
s.synchronize()
print("ok", n, "dense" if os.environ.get("DENSE", "0") == "1" else "smooth")
