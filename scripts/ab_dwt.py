"""ABBA A/B of the 2D-DWT encode variants (8 4K frames, l=5, bior4.4):
python scripts/ab_dwt.py 1,3"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,3").split(",")]
w = DW.wavelet_index(os.environ.get("WAVELET", "bior4.4"))
shapes, pb, wb = DW.layout(H, W, LV)
frames = np.stack([bench.synth_frame(H, W, s) for s in range(F)])
din, dws = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb)
outs = {v: DeviceBuffer(F * pb) for v in variants}
s = Stream()
DECODE = os.environ.get("DECODE", "0") == "1"
if DECODE:   # decode the default encode's subbands; outputs are RGB frames
    dpk = DeviceBuffer(F * pb)
    L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)
    Ho, Wo = 2 * shapes[0][0], 2 * shapes[0][1]
    nout = F * Ho * Wo * 3
    outs = {v: DeviceBuffer(nout) for v in variants}
    run = lambda v: L.dwt_decode_v(v, dpk.ptr, F, H, W, w, LV, Q, outs[v].ptr, dws.ptr,
                           s.handle)
else:
    nout = F * pb
    run = lambda v: L.dwt_encode_v(v, din.ptr, F, H, W, w, LV, Q, outs[v].ptr, dws.ptr,
                           s.handle)
for v in variants:
    run(v)
s.synchronize()
ref = outs[variants[0]].download(np.empty(nout, np.uint8))
for v in variants[1:]:
    print(f"variant {v} == variant {variants[0]}: "
          f"{np.array_equal(outs[v].download(np.empty(nout, np.uint8)), ref)}", flush=True)
for _ in range(300):   # past the clock ramp
    run(variants[0])
res = {v: [] for v in variants}
e0, e1 = Event(), Event()
for rnd in range(16):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        e0.record(s)
        for _ in range(10):
            run(v)
        e1.record(s)
        s.synchronize()
        res[v].append(e0.elapsed_ms(e1) / 10)
base = np.array(res[variants[0]])
for v in variants:
    print(f"dwt {'decode' if DECODE else 'encode'} variant {v}: median {np.median(res[v]):.4f} ms per {F} 4K frames; "
          f"per-round ratio to {variants[0]}: {np.median(np.array(res[v]) / base):.4f}", flush=True)
