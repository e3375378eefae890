"""C3 encode per-frame time vs batch size and schedule (variant 0 = two-chunk pipeline,
17 = one stream): python scripts/dwt_batch_scan.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
H, W, LV, Q = 2160, 3840, 5, 32
w = DW.wavelet_index("bior4.4")
shapes, pb, wb = DW.layout(H, W, LV)
FM = 16
frames = np.stack([bench.synth_frame(H, W, s % 4) for s in range(FM)])
din, dws, dout = DeviceBuffer.from_array(frames), DeviceBuffer(FM * wb), DeviceBuffer(FM * pb)
s = Stream()
e0, e1 = Event(), Event()
run = lambda v, n: L.dwt_encode_v(v, din.ptr, n, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)
for _ in range(200):
    run(0, 8)
for n in (1, 2, 4, 8, 16):
    for v in (17, 0):
        ts = []
        for rnd in range(6):
            e0.record(s)
            for _ in range(max(2, 40 // n)):
                run(v, n)
            e1.record(s)
            s.synchronize()
            ts.append(e0.elapsed_ms(e1) / max(2, 40 // n))
        t = float(np.median(ts))
        print(f"n={n:2d} variant {v:2d}: {t:.4f} ms per call, {t / n * 8:.4f} ms per 8 frames", flush=True)
