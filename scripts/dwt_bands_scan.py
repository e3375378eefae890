"""The C3 encode (8 4K frames, l=5, bior4.4, Q=32) for several band cuts of the fused
levels 1 + 2 kernel (VCF_DWT_BANDS: bands, read at each launch; 0 = the library's
cost model) -- or with WHAT=decode the C3 decode for several cuts of the inverse
2 + 1 kernel (VCF_IDWT21_BROWS: level-1 rows per band; WHAT=decode_line: VCF_IDWT_BANDS, bands of the
inverse line kernels of levels 3..5; WHAT=decode_pipe: VCF_DWT_DEC_PIPE 0 / 1, the decode on
one stream or as the two-chunk frame pipeline; WHAT=encode_pipe: VCF_DWT_ENC_PIPE likewise for
the encode) -- interleaved over R rounds
of N launches, HIP events; output checksums compared (the cut never changes a byte).
python scripts/dwt_bands_scan.py [N] [R] [cuts...]"""
import json
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device
from vcf_amd.synthetic import synth_frame

set_device(0)
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
cuts = [int(c) for c in sys.argv[3:]] or [0, 1, 2, 3, 4, 6, 8]
w = DW.wavelet_index("bior4.4")
_, pb, wb = DW.layout(H, W, LV)
frames = np.stack([synth_frame(H, W, s) for s in range(F)])
din, dws, dpk = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb), DeviceBuffer(F * pb)
s = Stream()


WHAT = os.environ.get("WHAT", "encode")
KNOB = {"encode": "VCF_DWT_BANDS", "decode": "VCF_IDWT21_BROWS", "decode_line": "VCF_IDWT_BANDS",
        "decode_pipe": "VCF_DWT_DEC_PIPE", "encode_pipe": "VCF_DWT_ENC_PIPE"}[WHAT]
dout = DeviceBuffer(F * H * W * 3)
L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)


def enc():
    if WHAT.startswith("encode"):
        L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)
    else:
        L.call("vcf_dwt_dz_decode", dpk.ptr, F, H, W, w, LV, Q, dout.ptr, dws.ptr, s.handle)


def setcut(c):
    if c or WHAT.endswith("_pipe"):   # (*_pipe: 0 = one stream, 1 = the two-chunk pipeline)
        os.environ[KNOB] = str(c)
    else:
        os.environ.pop(KNOB, None)


res, crc = {c: [] for c in cuts}, {}
for c in cuts:
    setcut(c)
    for _ in range(20):
        enc()
    s.synchronize()
    enc_side = WHAT.startswith("encode")
    crc[c] = zlib.crc32((dpk if enc_side else dout).download(
        np.empty(F * pb if enc_side else F * H * W * 3, np.uint8)).tobytes())
for r in range(R):
    for c in (cuts if r % 2 == 0 else cuts[::-1]):
        setcut(c)
        e0, e1 = Event(), Event()
        e0.record(s)
        for _ in range(n):
            enc()
        e1.record(s)
        s.synchronize()
        res[c].append(e0.elapsed_ms(e1) / n)
print(json.dumps({"what": f"C3 {WHAT} ms per 8 x 4K by band cut ({KNOB}; 0 = cost model)",
                  "same_bytes": len(set(crc.values())) == 1,
                  "ms_median": {str(c): round(float(np.median(v)), 4) for c, v in res.items()}}), flush=True)
