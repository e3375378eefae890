"""Diagnostic: deflate the C4 workload once, dump every strip's size and a
checksum of its bytes, and list the strips that differ from zlib.  ZLIB_SO:
a diagnostic build (scripts/libvcf_zprof_NAME.so) instead of the product library."""
import ctypes, sys, os, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vcf_amd.synthetic import synth_frame, c4_frame
from vcf_amd import _lib as L, dct
from vcf_amd.codec.tiff import strip_layout
from vcf_amd.device import DeviceBuffer, Stream
n, H, W = int(sys.argv[1]), 1080, 1920
bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
frames = np.concatenate([dct.encode(np.stack([c4_frame(bases, i) for i in range(f, min(n, f + 16))]), Q=32)
                         for f in range(0, n, 16)])
flat = np.ascontiguousarray(frames.reshape(n, -1))
fb = flat.shape[1]; _, _, sb = strip_layout(frames.shape[1:], 1)
spf = int(L.lib().vcf_zlib_strip_count(fb, sb)); total = spf * n; slot = int(L.lib().vcf_zlib_bound(sb))
d = DeviceBuffer.from_array(flat); out = DeviceBuffer(total * slot); sizes = DeviceBuffer(total * 4)
so = os.environ.get("ZLIB_SO")
if so:   # the workspace as the library under test sizes it
    P = ctypes.CDLL(os.path.join(ROOT, "scripts", "debug", so))
    P.vcf_zlib_workspace.restype = ctypes.c_int64
    P.vcf_zlib_workspace.argtypes = [ctypes.c_int64]
    ws = DeviceBuffer(int(P.vcf_zlib_workspace(total)))
else:
    ws = DeviceBuffer(int(L.lib().vcf_zlib_workspace(total)))
st = Stream()
if "ZFILL" in os.environ:   # the workspace's contents before the call (uninitialised-read probe)
    ws.fill(int(os.environ["ZFILL"]), st)
    st.synchronize()
from vcf_amd.device import Event
if so:
    P.vcf_zlib_strips.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    for rep in range(2):   # the second call timed
        e0, e1 = Event(), Event()
        e0.record(st)
        assert P.vcf_zlib_strips(d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle) == 0
        e1.record(st)
        st.synchronize()
    print(f"{so}: {e0.elapsed_ms(e1):.1f} ms", flush=True)
    if hasattr(P, "vcf_zlib_dbg_read"):
        st.synchronize()
        dbg = (ctypes.c_uint * 8)()
        P.vcf_zlib_dbg_read(dbg)
        print("window check:", list(dbg), flush=True)
else:
    L.call("vcf_zlib_strips", d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle)
st.synchronize()
sz = sizes.download(np.empty(total, np.int32))
o = out.download(np.empty(total * slot, np.uint8))
crc = np.array([zlib.crc32(o[s * slot:s * slot + sz[s]].tobytes()) for s in range(total)], np.uint32)
np.savez(sys.argv[2], sz=sz, crc=crc)
bad = [s for s in range(total) if o[s * slot:s * slot + sz[s]].tobytes() !=
       zlib.compress(flat[s // spf, (s % spf) * sb:(s % spf + 1) * sb].tobytes(), 6)]
print(f"{sys.argv[2]} ({so or 'product'}): total {total}, bad {len(bad)}: {bad[:40]}", flush=True)
sys.path.insert(0, os.path.join(ROOT, "scripts", "debug"))
from ztokens import first_divergence


def lazy_of(strip):   # K1's parse-order rule: distinct hashes per 64-position group
    b = strip.astype(np.uint32)
    h = ((b[:-2] << 10) ^ (b[1:-1] << 5) ^ b[2:]) & 0x7fff
    d = sum(len(np.unique(h[i:i + 64])) for i in range(0, len(h), 64))
    return d * 4 < len(h)


dump = {}
for b in bad[:6]:
    g = o[b * slot:b * slot + sz[b]].tobytes()
    src = flat[b // spf, (b % spf) * sb:(b % spf + 1) * sb]
    w = zlib.compress(src.tobytes(), 6)
    d = next((i for i in range(min(len(g), len(w))) if g[i] != w[i]), None)
    try:
        fd = first_divergence(g, w)
    except Exception as e:   # a corrupt stream
        fd = f"gpu stream does not parse: {e!r}"
    print(f"  strip {b}: gpu {len(g)} B, zlib {len(w)} B, first difference at byte {d}, lazy {lazy_of(src)}, "
          f"{fd}", flush=True)
    dump[f"src_{b}"] = src
    dump[f"gpu_{b}"] = np.frombuffer(g, np.uint8)
if dump:
    np.savez(sys.argv[2].replace(".npz", "_bad.npz"), **dump)
