"""Run the 2D-DWT encode (8 4K frames, l=5, bior4.4) N times with one variant: for rocprofv3 --pmc passes.
python scripts/dwt_once.py VARIANT [N]   (DECODE=1: the decode of those frames' subbands;
LIFT=1: the opt-in lifting entry points instead of VARIANT)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from vcf_amd import synthetic as bench
import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Stream, set_device

set_device(0)
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
v = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = DW.wavelet_index(os.environ.get("WAVELET", "bior4.4"))
_, pb, wb = DW.layout(H, W, LV)
frames = np.stack([bench.synth_frame(H, W, s) for s in range(F)])
din, dws, dout = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb), DeviceBuffer(F * pb)
s = Stream()
if os.environ.get("LIFT", "0") == "1":
    def enc(*a):
        L.call("vcf_dwt_dz_encode_lift", *a[1:])

    def dec(*a):
        L.call("vcf_dwt_dz_decode_lift", *a[1:])
else:
    enc, dec = L.dwt_encode_v, L.dwt_decode_v
if os.environ.get("DECODE", "0") == "1":
    L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)
    for _ in range(n):
        dec(v, dout.ptr, F, H, W, w, LV, Q, din.ptr, dws.ptr, s.handle)
else:
    for _ in range(n):
        enc(v, din.ptr, F, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)
s.synchronize()
print("ok", v, n)
