"""Prior classes (container version 3) vs one prior (version 2): single-frame
GPU encode / decode latency and rate of the tiled CBAAC on DCT indices, and
batch throughput (FrameBatch).  python scripts/bench_tcbaac_classes.py -> JSON lines.

Timed: the kernels on device-resident indices (prior rows + encode; decode
from the payload in HBM), HIP events on the coder's stream, median of reps.
Rate: the container bytes (prior rows included) over the host serial coder's
stream of the same indices (vcf_cbaac_encode, the reference's algorithm)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd._lib as L
from oracle import oracle as O
from vcf_amd import tcbaac as T
from vcf_amd.cbaac import encode_symbols
from vcf_amd.device import DeviceBuffer, Event, set_device


def timed(fn, stream, reps=7):
    fn()
    stream.synchronize()
    ts = []
    for _ in range(reps):
        a, b = Event(), Event()
        a.record(stream)
        fn()
        b.record(stream)
        b.synchronize()
        ts.append(a.elapsed_ms(b))
    return float(np.median(ts))


def single(k, shape, seg, K):
    n = k.size
    c = T.TiledCoder(0, seg, prior=True, nclass=K)
    st = c.stream
    sym = DeviceBuffer.from_array(k)
    sizes, payload = c.encode_device(sym, n)
    prior = c.last_prior
    data = T.pack(shape, 0, seg, sizes, payload, prior)
    lib = L.lib()
    ns = T.n_segments(n, seg)
    ws = c.scratch.get("ws", int(lib.vcf_cbaac_tiled_workspace(n, seg)))
    cap = int(lib.vcf_cbaac_tiled_bound(n, seg))
    ob, sb = c.scratch.get("out", cap), c.scratch.get("sizes", 8 * (ns + 1))
    pr, hist = c.scratch.get("prior", 512 * K), c.scratch.get("hist", 1024 * K)

    def enc():
        if K > 1:
            L.call("vcf_cbaac_tiled_prior_classes", sym.ptr, 1, n, n, seg, K, pr.ptr, hist.ptr, st.handle)
            L.call("vcf_cbaac_tiled_encode_classes", sym.ptr, 1, n, n, 0, pr.ptr, K, seg, ob.ptr, cap, sb.ptr, ws.ptr,
                   st.handle)
        else:
            L.call("vcf_cbaac_tiled_prior", sym.ptr, n, pr.ptr, hist.ptr, st.handle)
            L.call("vcf_cbaac_tiled_encode_prior", sym.ptr, n, 0, pr.ptr, seg, ob.ptr, cap, sb.ptr, ws.ptr, st.handle)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    src, doffs = DeviceBuffer.from_array(np.frombuffer(payload, np.uint8)), DeviceBuffer.from_array(offs)
    dpr = DeviceBuffer.from_array(np.ascontiguousarray(prior))
    out = DeviceBuffer(n)

    def dec():
        if K > 1:
            L.call("vcf_cbaac_tiled_decode_classes", src.ptr, doffs.ptr, 1, n, 0, dpr.ptr, K, seg, out.ptr, n, st.handle)
        else:
            L.call("vcf_cbaac_tiled_decode_prior", src.ptr, doffs.ptr, n, 0, dpr.ptr, seg, out.ptr, st.handle)
    e_ms, d_ms = timed(enc, st), timed(dec, st)
    ok = np.array_equal(out.download(np.empty(n, np.uint8)), k)
    return e_ms, d_ms, len(data), ns, ok


def main():
    set_device(0)
    for (H, W) in ((1080, 1920), (2160, 3840)):
        k = np.ascontiguousarray(O.encode_frame(bench.synth_frame(H, W, 0), 32, 0))
        shape = k.shape
        k = k.ravel()
        serial = len(encode_symbols(k, 0))
        for seg, K in ((32768, 1), (4096, 1), (2048, 8), (4096, 8), (8192, 8)):
            e_ms, d_ms, nbytes, ns, ok = single(k, shape, seg, K)
            print(json.dumps(dict(case="tcbaac_single_frame", frame=[H, W, 3], seg_len=seg, nclass=K, segments=ns,
                                  encode_ms=round(e_ms, 3), decode_ms=round(d_ms, 3), container_bytes=nbytes,
                                  serial_bytes=serial, rate_overhead=round(nbytes / serial - 1, 4), round_trip=ok)),
                  flush=True)
    k = np.ascontiguousarray(O.encode_frame(bench.synth_frame(1080, 1920, 0), 32, 0)).ravel()
    for F in (16, 256):
        frames = np.tile(k, F)
        buf = DeviceBuffer.from_array(frames)
        for seg, K in ((32768, 1), (4096, 8)):
            fb = T.FrameBatch(F, k.size, 0, seg, prior=True, nclass=K)
            ms = timed(lambda: fb.launch(buf), fb.stream, 3)
            print(json.dumps(dict(case="tcbaac_frames", frames=F, frame=[1080, 1920, 3], seg_len=seg, nclass=K,
                                  encode_ms=round(ms, 2), Gsym_s=round(F * k.size / ms / 1e6, 2))), flush=True)


if __name__ == "__main__":
    main()
