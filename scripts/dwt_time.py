"""Time the C3 DWT encode and decode (8 4K frames, l=5, bior4.4, Q=32) through
whichever library VCF_AMD_LIB names: median ms of R rounds of N launches, HIP
events on the launch stream.  For A/B runs (ABBA across library builds).
python scripts/dwt_time.py [N] [R]   (LIFT=1: the lifting entry points)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from vcf_amd import synthetic as bench
import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
sfx = "_lift" if os.environ.get("LIFT", "0") == "1" else ""
w = DW.wavelet_index("bior4.4")
_, pb, wb = DW.layout(H, W, LV)
frames = np.stack([bench.synth_frame(H, W, s) for s in range(F)])
din, dws, dpk = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb), DeviceBuffer(F * pb)
dout = DeviceBuffer(F * H * W * 3)
s = Stream()
enc = lambda: L.call("vcf_dwt_dz_encode" + sfx, din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)  # noqa
dec = lambda: L.call("vcf_dwt_dz_decode" + sfx, dpk.ptr, F, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)  # noqa
out = {"lib": os.environ.get("VCF_AMD_LIB", "product")}
for name, fn in (("encode", enc), ("decode", dec)):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(R):
        e0, e1 = Event(), Event()
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        s.synchronize()
        ts.append(e0.elapsed_ms(e1) / n)
    out[name] = round(float(np.median(ts)), 4)
enc()
s.synchronize()
out["packed_crc"] = int(np.frombuffer(dpk.download(np.empty(F * pb, np.uint8)), np.uint64).sum() % (1 << 61))
dec()
s.synchronize()
out["rgb_crc"] = int(np.frombuffer(dout.download(np.empty(F * H * W * 3, np.uint8)), np.uint64).sum() % (1 << 61))
print(json.dumps(out))
