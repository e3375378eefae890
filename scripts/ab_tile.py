"""Encode-kernel tile-size A/B (VCF_ENC_TILE = 256 / 384 / 512, read once per
process): 64 x 4K S-smooth frames per launch, settled clocks, event-timed
launches; prints ms per launch and a CRC of the output (must match across tiles)."""
import json, os, sys, time, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import synth_frame
from vcf_amd import dct as D
from vcf_amd.device import DeviceBuffer, Event, Stream
H, W, F = 2160, 3840, 64
fr = [synth_frame(H, W, s) for s in range(4)]
din = DeviceBuffer(F * H * W * 3)
for f in range(F):
    din.upload(fr[f % 4], offset=f * H * W * 3)
dout = DeviceBuffer(F * H * W * 3)
st = Stream()
step = lambda: D.encode_device(din, F, H, W, 32, 0, out=dout, stream=st)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for _ in range(20):
        step()
    st.synchronize()
e0, e1 = Event(), Event()
e0.record(st)
for _ in range(200):
    step()
e1.record(st)
st.synchronize()
k = dout.download(np.empty(F * H * W * 3, np.uint8))
print(json.dumps({"tile": os.environ.get("VCF_ENC_TILE", "256"), "ms": round(e0.elapsed_ms(e1) / 200, 4),
                  "crc": zlib.crc32(k[: 8 * H * W * 3].tobytes())}), flush=True)
