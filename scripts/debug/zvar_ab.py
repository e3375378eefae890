"""ABBA timing of GPU deflate variants (scripts/debug/zvar_build.sh builds) against
the product library on the C4 workload, one process: the call is timed with HIP
events, variants alternate order each round, every variant's strips are checked
equal to the product's (and the product's first frame to zlib).
    python scripts/debug/zvar_ab.py N_FRAMES ROUNDS NAME...   (libvcf_zvar_NAME.so)"""
import ctypes
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vcf_amd import _lib as L, dct   # noqa: E402
from vcf_amd.codec.tiff import strip_layout   # noqa: E402
from vcf_amd.device import DeviceBuffer, Event, Stream   # noqa: E402
from vcf_amd.synthetic import c4_frame, synth_frame   # noqa: E402

n, R, names = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
H, W = 1080, 1920
bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
frames = np.concatenate([dct.encode(np.stack([c4_frame(bases, i) for i in range(f, min(n, f + 16))]), Q=32)
                         for f in range(0, n, 16)])
flat = np.ascontiguousarray(frames.reshape(n, -1))
fb = flat.shape[1]
sb = strip_layout(frames.shape[1:], 1)[2]
spf = int(L.lib().vcf_zlib_strip_count(fb, sb))
total, slot = spf * n, int(L.lib().vcf_zlib_bound(sb))
d, sizes = DeviceBuffer.from_array(flat), DeviceBuffer(total * 4)
st = Stream()
libs = {"product": L.lib()}
for nm in names:
    P = ctypes.CDLL(os.path.join(ROOT, "scripts", "debug", f"libvcf_zvar_{nm}.so"))
    P.vcf_zlib_strips.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    P.vcf_zlib_workspace.restype = ctypes.c_int64
    P.vcf_zlib_workspace.argtypes = [ctypes.c_int64]
    libs[nm] = P
ws = DeviceBuffer(max(int(P.vcf_zlib_workspace(total)) for P in libs.values()))
outs = {k: DeviceBuffer(total * slot) for k in libs}


def run(k):
    rc = libs[k].vcf_zlib_strips(d.ptr, n, fb, sb, 6, outs[k].ptr, slot, sizes.ptr, ws.ptr, st.handle)
    assert rc == 0, (k, rc)


res, got = {k: [] for k in libs}, {}
for k in libs:   # warm-up and outputs
    run(k)
    st.synchronize()
    sz = sizes.download(np.empty(total, np.int32))
    o = outs[k].download(np.empty(total * slot, np.uint8))
    got[k] = [o[s * slot:s * slot + sz[s]].tobytes() for s in range(total)]
ok_zlib = all(got["product"][s] == zlib.compress(flat[0, s * sb:(s + 1) * sb].tobytes(), 6) for s in range(spf))
same = {k: got[k] == got["product"] for k in libs}
order = list(libs)
for r in range(R):
    for k in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = Event(), Event()
        e0.record(st)
        run(k)
        e1.record(st)
        st.synchronize()
        res[k].append(e0.elapsed_ms(e1))
print(json.dumps({"frames": n, "strips": total, "product_frame0_equals_zlib": ok_zlib, "same_bytes": same,
                  "ms_median": {k: round(float(np.median(v)), 2) for k, v in res.items()},
                  "ms_all": {k: [round(x, 2) for x in v] for k, v in res.items()}}), flush=True)
