"""ABBA of a process-wide switch of the C3 DWT path (8 4K frames, l=5, bior4.4,
Q=32): python scripts/dwt_toggle_ab.py SETTER [decode|encode] [rounds]
e.g. vcf_dwt_set_inverse_band21 decode.  Median ms per launch per setting (HIP
events on the launch stream), and both settings' output checksums."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device
from vcf_amd.synthetic import synth_frame

set_device(0)
setter = sys.argv[1]
what = sys.argv[2] if len(sys.argv) > 2 else "decode"
R = int(sys.argv[3]) if len(sys.argv) > 3 else 12
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
w = DW.wavelet_index(os.environ.get("WAVELET", "bior4.4"))
_, pb, wb = DW.layout(H, W, LV)
frames = np.stack([synth_frame(H, W, s) for s in range(F)])
din, dws, dpk = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb), DeviceBuffer(F * pb)
dout = DeviceBuffer(F * H * W * 3)
s = Stream()
enc = lambda: L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)  # noqa
dec = lambda: L.call("vcf_dwt_dz_decode", dpk.ptr, F, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)  # noqa
fn = dec if what == "decode" else enc
enc()
res, crc = {0: [], 1: []}, {}
for v in (1, 0):
    L.call(setter, v)
    for _ in range(20):
        fn()
    s.synchronize()
    buf = dout if what == "decode" else dpk
    crc[v] = int(np.frombuffer(buf.download(np.empty(buf.nbytes, np.uint8)), np.uint64).sum() % (1 << 61))
for r in range(R):
    for v in ((1, 0) if r % 2 == 0 else (0, 1)):
        L.call(setter, v)
        e0, e1 = Event(), Event()
        e0.record(s)
        for _ in range(20):
            fn()
        e1.record(s)
        s.synchronize()
        res[v].append(e0.elapsed_ms(e1) / 20)
L.call(setter, 1)
print(json.dumps({"setter": setter, "what": what, "ms_on": round(float(np.median(res[1])), 4),
                  "ms_off": round(float(np.median(res[0])), 4), "crc_on": crc[1], "crc_off": crc[0],
                  "same_bytes": crc[0] == crc[1]}))
