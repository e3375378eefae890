"""A/B the encode kernel variants in one process (interleaved rounds, §5.4 rule 24)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd.dct as D
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
H, W, F, Q = 2160, 3840, 64, 32
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2"])]
Hp, Wp = D.padded_shape(H, W)
frames = [bench.synth_frame(H, W, s) for s in range(4)]
din = DeviceBuffer(F * H * W * 3)
for f in range(F):
    din.upload(frames[f % 4], offset=f * H * W * 3)
outs = {v: DeviceBuffer(F * Hp * Wp * 3) for v in variants}
s = Stream()
for v in variants:
    D.encode_device(din, F, H, W, Q, out=outs[v], stream=s, variant=v)
s.synchronize()
ref = outs[variants[0]].download(np.empty((F, Hp, Wp, 3), np.uint8))
for v in variants[1:]:
    if v in (2, 6, 8):
        continue   # diagnostic variants do not produce the output
    o = outs[v].download(np.empty((F, Hp, Wp, 3), np.uint8))
    print(f"variant {v} == variant {variants[0]}: {np.array_equal(o, ref)}", flush=True)
res = {v: [] for v in variants}
e0, e1 = Event(), Event()
ROUNDS = int(os.environ.get("ROUNDS", "16"))
for rnd in range(ROUNDS):
    order = variants if rnd % 2 == 0 else variants[::-1]   # ABBA: cancel position effects
    for v in order:
        e0.record(s)
        for _ in range(10):
            D.encode_device(din, F, H, W, Q, out=outs[v], stream=s, variant=v)
        e1.record(s)
        s.synchronize()
        res[v].append(e0.elapsed_ms(e1) / 10)
alg = F * (H * W * 3 + Hp * Wp * 3)
base = np.array(res[variants[0]])
for v in variants:
    t = np.median(res[v])
    ratio = np.median(np.array(res[v]) / base)
    print(f"variant {v}: median {t:.4f} ms/launch (min {min(res[v]):.4f}) -> "
          f"{alg / t / 1e6:.0f} GB/s ({alg / t / 1e6 / 8000:.1%} of 8 TB/s), "
          f"{F * H * W / t / 1e3:.0f} Mpix/s; per-round ratio to {variants[0]}: {ratio:.4f}", flush=True)
