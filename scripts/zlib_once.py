"""Deflate bench.py's C4 workload (n 1080p DCT index frames, shifted S-smooth
content) with vcf_zlib_strips R times, for rocprofv3 passes; the last call's
strips of frames 0 and n-1 are checked against zlib.compress.
    python scripts/zlib_once.py [n_frames=256] [reps=2]"""
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from vcf_amd import _lib as L
from vcf_amd import dct
from vcf_amd.codec.tiff import strip_layout
from vcf_amd.device import DeviceBuffer, Stream, set_device
from vcf_amd.synthetic import c4_frame, synth_frame

set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H, W = 1080, 1920
bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
frames = np.concatenate([dct.encode(np.stack([c4_frame(bases, i) for i in range(f, min(n, f + 16))]), Q=32)
                         for f in range(0, n, 16)])
flat = np.ascontiguousarray(frames.reshape(n, -1))
fb = flat.shape[1]
sb = strip_layout(frames.shape[1:], 1)[2]
spf = int(L.lib().vcf_zlib_strip_count(fb, sb))
total, slot = spf * n, int(L.lib().vcf_zlib_bound(sb))
d, out, sizes = DeviceBuffer.from_array(flat), DeviceBuffer(total * slot), DeviceBuffer(total * 4)
ws = DeviceBuffer(int(L.lib().vcf_zlib_workspace(total)))
st = Stream()
for _ in range(reps):
    L.call("vcf_zlib_strips", d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle)
st.synchronize()
sz = sizes.download(np.empty(total, np.int32))
o = out.download(np.empty(total * slot, np.uint8))
chk = list(range(spf)) + list(range((n - 1) * spf, total))
bad = [s for s in chk if o[s * slot:s * slot + sz[s]].tobytes() !=
       zlib.compress(flat[s // spf, (s % spf) * sb:(s % spf + 1) * sb].tobytes(), 6)]
print(f"zlib_once: {n} frames, {total} strips, {reps} calls, {int(sz.sum())} bytes, bad {len(bad)} of {len(chk)} "
      "checked", flush=True)
sys.exit(1 if bad else 0)
