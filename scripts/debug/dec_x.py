import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, bench, vcf_amd.dct as D
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device
set_device(0)
H, W, F, Q = 2160, 3840, 64, 32
din = DeviceBuffer(F * H * W * 3)
fr = bench.synth_frame(H, W, 0)
for f in range(F): din.upload(fr, offset=f * H * W * 3)
s = Stream(); e0, e1 = Event(), Event()
for flags in (0, 1, 0, 1):
    dk = DeviceBuffer(F * H * W * 3); out = DeviceBuffer(F * H * W * 3)
    D.encode_device(din, F, H, W, Q, flags, out=dk, stream=s)
    for _ in range(5): D.decode_device(dk, F, H, W, Q, flags, out=out, stream=s)
    e0.record(s)
    for _ in range(20): D.decode_device(dk, F, H, W, Q, flags, out=out, stream=s)
    e1.record(s); s.synchronize()
    print("flags", flags, "decode ms", e0.elapsed_ms(e1) / 20, flush=True)
