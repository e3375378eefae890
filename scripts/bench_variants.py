"""A/B the encode (or, with DECODE=1, the decode) kernel variants in one process
(interleaved ABBA rounds, §5.4 rule 24).  Variant 0 is the product library's
kernel, the others the A/B library's (include/vcf_amd_ab.h).  DENSE=1: uniform
random frames instead of S-smooth (every coefficient nonzero: the decode's
worst case)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd.dct as D
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
H, W, F, Q = 2160, 3840, 64, 32
DECODE = os.environ.get("DECODE", "0") == "1"
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2"])]
Hp, Wp = D.padded_shape(H, W)
if os.environ.get("DENSE", "0") == "1":
    frames = [np.random.Generator(np.random.PCG64(s)).integers(0, 256, (H, W, 3), dtype=np.uint8) for s in range(4)]
else:
    frames = [bench.synth_frame(H, W, s) for s in range(4)]
din = DeviceBuffer(F * H * W * 3)
for f in range(F):
    din.upload(frames[f % 4], offset=f * H * W * 3)
s = Stream()
if DECODE:
    dk = DeviceBuffer(F * Hp * Wp * 3)
    D.encode_device(din, F, H, W, Q, out=dk, stream=s)
    outs = {v: DeviceBuffer(F * H * W * 3) for v in variants}
    run = lambda v: D.decode_device(dk, F, H, W, Q, out=outs[v], stream=s, variant=v)
    oshape = (F, H, W, 3)
    diag = ()
else:
    outs = {v: DeviceBuffer(F * Hp * Wp * 3) for v in variants}
    run = lambda v: D.encode_device(din, F, H, W, Q, out=outs[v], stream=s, variant=v)
    oshape = (F, Hp, Wp, 3)
    diag = (2, 6, 8, 9, 10)   # diagnostic variants do not produce the output
for v in variants:
    run(v)
s.synchronize()
ref = outs[variants[0]].download(np.empty(oshape, np.uint8))
for v in variants[1:]:
    if v in diag:
        continue
    o = outs[v].download(np.empty(oshape, np.uint8))
    print(f"variant {v} == variant {variants[0]}: {np.array_equal(o, ref)}", flush=True)
res = {v: [] for v in variants}
e0, e1 = Event(), Event()
ROUNDS = int(os.environ.get("ROUNDS", "16"))
for rnd in range(ROUNDS):
    order = variants if rnd % 2 == 0 else variants[::-1]   # ABBA: cancel position effects
    for v in order:
        e0.record(s)
        for _ in range(10):
            run(v)
        e1.record(s)
        s.synchronize()
        res[v].append(e0.elapsed_ms(e1) / 10)
alg = F * (H * W * 3 + Hp * Wp * 3)
base = np.array(res[variants[0]])
for v in variants:
    t = np.median(res[v])
    ratio = np.median(np.array(res[v]) / base)
    print(f"{'decode' if DECODE else 'encode'} variant {v}: median {t:.4f} ms/launch (min {min(res[v]):.4f}) -> "
          f"{alg / t / 1e6:.0f} GB/s ({alg / t / 1e6 / 8000:.1%} of 8 TB/s), "
          f"{F * H * W / t / 1e3:.0f} Mpix/s; per-round ratio to {variants[0]}: {ratio:.4f}", flush=True)
