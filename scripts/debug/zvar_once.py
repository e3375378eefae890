"""One variant library's vcf_zlib_strips on the C4 workload, R times, for rocprofv3
kernel traces of diagnostic builds (scripts/debug/zvar_build.sh).
    python scripts/debug/zvar_once.py NAME [n_frames=256] [reps=2]   (libvcf_zvar_NAME.so)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vcf_amd import _lib as L, dct   # noqa: E402
from vcf_amd.codec.tiff import strip_layout   # noqa: E402
from vcf_amd.device import DeviceBuffer, Stream   # noqa: E402
from vcf_amd.synthetic import c4_frame, synth_frame   # noqa: E402

name = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
bases = [synth_frame(1080, 1920, seed=100 + s) for s in range(4)]
frames = np.concatenate([dct.encode(np.stack([c4_frame(bases, i) for i in range(f, min(n, f + 16))]), Q=32)
                         for f in range(0, n, 16)])
flat = np.ascontiguousarray(frames.reshape(n, -1))
fb = flat.shape[1]
sb = strip_layout(frames.shape[1:], 1)[2]
P = ctypes.CDLL(os.path.join(ROOT, "scripts", "debug", f"libvcf_zvar_{name}.so"))
P.vcf_zlib_strips.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
P.vcf_zlib_workspace.restype = ctypes.c_int64
P.vcf_zlib_workspace.argtypes = [ctypes.c_int64]
spf = int(L.lib().vcf_zlib_strip_count(fb, sb))
total, slot = spf * n, int(L.lib().vcf_zlib_bound(sb))
d, sizes, out = DeviceBuffer.from_array(flat), DeviceBuffer(total * 4), DeviceBuffer(total * slot)
ws = DeviceBuffer(int(P.vcf_zlib_workspace(total)))
st = Stream()
for _ in range(reps):
    assert P.vcf_zlib_strips(d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle) == 0
st.synchronize()
print("ok", name, total)
