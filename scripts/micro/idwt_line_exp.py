"""A/B of level-1 line-inverse kernels on config C3 (8 4K frames, bior4.4, l=5,
Q=32): the product decode (variant 17) leaves level 2's output plane (LL1) in
the workspace; each experimental kernel rebuilds the RGB frames from it and the
level-1 subbands, checked byte for byte against the product decode.
python scripts/micro/idwt_line_exp.py VARIANTS [BANDS,...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np

import bench
import vcf_amd._lib as L
import vcf_amd.dwt as DW
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

set_device(0)
exp = ctypes.CDLL(os.path.join(ROOT, "scripts/micro/libidwt_line_exp.so"))
H, W, F, LV, Q = 2160, 3840, 8, 5, 32
variants = [int(v) for v in sys.argv[1].split(",")]
bands = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "4").split(",")]
w = DW.wavelet_index("bior4.4")
shapes, pb, wb = DW.layout(H, W, LV)
frames = np.stack([bench.synth_frame(H, W, s) for s in range(F)])
din, dws, dpk = DeviceBuffer.from_array(frames), DeviceBuffer(F * wb), DeviceBuffer(F * pb)
s = Stream()
L.call("vcf_dwt_dz_encode", din.ptr, F, H, W, w, LV, Q, dpk.ptr, dws.ptr, s.handle)
ref = DeviceBuffer(F * H * W * 3)
L.dwt_decode_v(17, dpk.ptr, F, H, W, w, LV, Q, ref.ptr, dws.ptr, s.handle)
s.synchronize()
want = ref.download(np.empty(F * H * W * 3, np.uint8))
hs = [H] + [h for h, _ in shapes]
ws = [W] + [x for _, x in shapes]
off = 2 * hs[LV] * ws[LV] * 3
sb = {}
for r in range(LV, 0, -1):
    sb[r] = []
    for _ in range(3):
        sb[r].append(off)
        off += 3 * hs[r] * ws[r]
col, inv, ll = hs[1] * ws[0], hs[1] * 2 * ws[1], 2 * hs[1] * 2 * ws[1]
pd = 2 * max(col, inv) + 2 * ll
D0 = max(hs[1] * ws[0], hs[1] * 2 * ws[1])
P0 = 2 * D0
P1 = P0 + 4 * hs[1] * ws[1]
prev = ctypes.c_void_p(dws.ptr.value + 8 * P1)
out = DeviceBuffer(F * H * W * 3)
h1, w1 = hs[1], ws[1]
for nb in bands:
    for v in variants:
        run = lambda: exp.exp_line_l1(v, dpk.ptr, ctypes.c_longlong(pb), ctypes.c_longlong(sb[1][0]),
                                      ctypes.c_longlong(sb[1][1]), ctypes.c_longlong(sb[1][2]), prev,
                                      ctypes.c_longlong(pd), ws[1], out.ptr, h1, w1, 2 * h1, 2 * w1, Q, F, nb,
                                      s.handle)
        out.fill(0, s)
        assert run() == 0
        s.synchronize()
        got = out.download(np.empty_like(want))
        ok = bool(np.array_equal(got, want))
        e0, e1 = Event(), Event()
        for _ in range(3):
            run()
        e0.record(s)
        for _ in range(20):
            run()
        e1.record(s)
        s.synchronize()
        print(f"variant {v} bands {nb}: {e0.elapsed_ms(e1) / 20:.4f} ms  equal={ok}", flush=True)
