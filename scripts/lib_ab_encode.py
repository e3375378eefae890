"""ABBA of a hot path between the product library and variant libraries built by
scripts/build_variant.sh, in one process: each library loaded with ctypes,
launches timed with HIP events on one stream, the order alternating per round;
outputs compared byte for byte.
    python scripts/lib_ab_encode.py ROUNDS NAME...   (vcf_amd/libvcf_amd_NAME.so)
WHAT=encode (default): the headline encode, 64 4K frames, Q=32 (dct_dz_encode);
WHAT=dwtdec: the C3 2D-DWT decode, 8 4K frames, l=5 bior4.4, Q=32."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vcf_amd import _lib as L   # noqa: E402
from vcf_amd import dct as D   # noqa: E402
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device   # noqa: E402
from vcf_amd.synthetic import synth_frame   # noqa: E402

set_device(0)
R, names = int(sys.argv[1]), sys.argv[2:]
WHAT = os.environ.get("WHAT", "encode")
H, W, F, Q = 2160, 3840, (64 if WHAT == "encode" else 8), 32
Hp, Wp = D.padded_shape(H, W)
frames = [synth_frame(H, W, s) for s in range(4)]
din = DeviceBuffer(F * H * W * 3)
for f in range(F):
    din.upload(frames[f % 4], offset=f * H * W * 3)
st = Stream()
libs = {"product": L.lib()}
for nm in names:
    P = ctypes.CDLL(os.path.join(ROOT, "vcf_amd", f"libvcf_amd_{nm}.so"))
    P.vcf_dct_dz_encode.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    P.vcf_dwt_dz_decode.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    libs[nm] = P
if WHAT == "encode":
    outs = {k: DeviceBuffer(F * Hp * Wp * 3) for k in libs}

    def run(k):
        assert libs[k].vcf_dct_dz_encode(din.ptr, F, H, W, 8, Q, 0, outs[k].ptr, st.handle) == 0
else:
    import vcf_amd.dwt as DW
    wv = DW.wavelet_index("bior4.4")
    _, pb, wb = DW.layout(H, W, 5)
    dpk, dws = DeviceBuffer(F * pb), DeviceBuffer(F * wb)
    DW.encode_device(din, F, H, W, wv, 5, Q, dpk, dws, st)
    outs = {k: DeviceBuffer(F * H * W * 3) for k in libs}

    def run(k):
        assert libs[k].vcf_dwt_dz_decode(dpk.ptr, F, H, W, wv, 5, Q, outs[k].ptr, dws.ptr, st.handle) == 0


for k in libs:
    for _ in range(200):   # past the clock ramp
        run(k)
st.synchronize()
ref = outs["product"].download(np.empty(outs["product"].nbytes, np.uint8))
same = {k: bool(np.array_equal(outs[k].download(np.empty_like(ref)), ref)) for k in libs}
res = {k: [] for k in libs}
order = list(libs)
for r in range(R):
    for k in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = Event(), Event()
        e0.record(st)
        for _ in range(50):
            run(k)
        e1.record(st)
        st.synchronize()
        res[k].append(e0.elapsed_ms(e1) / 50)
print(json.dumps({"what": f"{WHAT} ({F} x 4K), ms per launch", "same_bytes": same,
                  "ms_median": {k: round(float(np.median(v)), 4) for k, v in res.items()},
                  "ms_all": {k: [round(x, 4) for x in v] for k, v in res.items()}}), flush=True)
