"""Diagnostic: bench.py's C5 block on a short sequence, then its checker leg."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from vcf_amd.comm import HostGroup
a = argparse.Namespace(c5_frames=int(sys.argv[1]) if len(sys.argv) > 1 else 12, QSS=32, c5_steps=1, c5_warmup=0,
                       c4_timeout=120.0)
info = bench.c5_block(a, 1, 0, HostGroup(0, 1))
bench.c5_check(info, 32)
print(json.dumps(info)[:1500], flush=True)
# the same sequence through one DeviceIPP run, every frame against the oracle loop
import numpy as np
from oracle import oracle as O
from vcf_amd.codec.ipp_device import DeviceIPP
from vcf_amd.codec.tiff import imwrite_bytes
from vcf_amd.device import DeviceBuffer
N, H, W = a.c5_frames, 2160, 3840
base = bench.synth_frame(H + 48, W + 64, seed=500)
frames = [bench.c5_frame(base, i, H, W) for i in range(N)]
job = DeviceIPP(None, 0, 1, N, H, W, 32, 10, 16, 8, False)
for run in range(2):
    sizes, got, mvs = job.run(DeviceBuffer.from_array(np.stack(frames)))
    ks, want_mv = [], []
    k = O.encode_frame(frames[0], 32); ks.append(k); ref = O.decode_frame(k, H, W, 32)
    for p in range(1, min(3, N)):
        mv = O.ipp_block_matching(ref, frames[p], 16, 8, False)
        comp = O.ipp_motion_compensate(ref, mv, 16)
        k = O.encode_frame(O.ipp_residual(frames[p], comp), 32); ks.append(k)
        ref = O.ipp_reconstruct(comp, O.decode_frame(k, H, W, 32)); want_mv.append(mv)
    for i in range(len(ks)):
        w = imwrite_bytes(ks[i])
        print(f"run {run} frame {i}: file {'ok' if bytes(got[i]) == w else 'DIFF'} ({len(got[i])}/{len(w)})", flush=True)
    for i, m in enumerate(want_mv):
        g = np.asarray(mvs[i])
        print(f"run {run} mv {i + 1}: {'ok' if np.array_equal(g, m) else 'DIFF'} shapes {g.shape}/{m.shape} "
              f"dtypes {g.dtype}/{m.dtype} ndiff {int((g != m).sum()) if g.shape == m.shape else -1}", flush=True)
