"""C2 (1080p frame, YCoCg + 2D-DCT B=8 + deadzone + CBAAC) per-stage breakdown
of CoDec.encode_fn (vcf_amd/codec/dct2d.py:268-294), the stages timed one by
one with the same calls encode_fn makes:

  read     encode_read_fn: the PNG decode (native reader, codec/eic.py)
  h2d      DeviceBuffer.from_array of the RGB frame (pageable host memory)
  dct      vcf_dct_dz_encode on the GPU (indices stay in HBM)
  entropy  the tiled coder's kernels (TCBAACP: class histograms + prior rows, encode)
  d2h      segment sizes + code-stream bytes back to the host
  pack     the container (tcbaac.pack) + _shape.bin
  write    encode_write_fn (file write)

plus the whole encode_fn for comparison, for -c TCBAAC / TCBAACP (GPU coder)
and -c CBAAC (the reference's serial coder on the host: indices D2H, then
the native CPU coder).  python scripts/c2_stages.py [reps] -> JSON lines."""
import json
import os
import struct
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from PIL import Image

import bench
import vcf_amd._lib as L
import vcf_amd.dct as D
from vcf_amd.codec import parser as P
from vcf_amd.codec.dct2d import CoDec
from vcf_amd.device import DeviceBuffer, set_device
from vcf_amd.tcbaac import n_segments, pack


def med(xs):
    return round(float(np.median(xs)), 3)


def stages_gpu_coder(c, src, out, reps):
    ent = c.entropy
    coder = ent.coder
    st = coder.stream
    lib = L.lib()
    t = {k: [] for k in ("read", "h2d", "dct", "entropy", "d2h", "pack", "write")}
    for it in range(reps + 1):
        t0 = time.perf_counter()
        img = c.encode_read_fn(src)
        t1 = time.perf_counter()
        H, W = img.shape[:2]
        Hp, Wp = D.padded_shape(H, W, c.block_size)
        n = Hp * Wp * 3
        srcb = DeviceBuffer.from_array(img, st)
        st.synchronize()
        t2 = time.perf_counter()
        k = DeviceBuffer(n)
        D.encode_device(srcb, 1, H, W, c.QSS, c.flags, out=k, stream=st, block_size=c.block_size)
        st.synchronize()
        t3 = time.perf_counter()
        ns = n_segments(n, coder.seg_len)
        ws = coder.scratch.get("ws", int(lib.vcf_cbaac_tiled_workspace(n, coder.seg_len)))
        cap = int(lib.vcf_cbaac_tiled_bound(n, coder.seg_len))
        ob = coder.scratch.get("out", cap)
        sb = coder.scratch.get("sizes", 8 * (ns + 1))
        K = coder.nclass
        if coder.prior and K > 1:
            pr, hist = coder.scratch.get("prior", 512 * K), coder.scratch.get("hist", 1024 * K)
            L.call("vcf_cbaac_tiled_prior_classes", k.ptr, 1, n, n, coder.seg_len, K, pr.ptr, hist.ptr, st.handle)
            L.call("vcf_cbaac_tiled_encode_classes", k.ptr, 1, n, n, coder.order, pr.ptr, K, coder.seg_len, ob.ptr,
                   cap, sb.ptr, ws.ptr, st.handle)
        elif coder.prior:
            pr, hist = coder.scratch.get("prior", 512), coder.scratch.get("hist", 1024)
            L.call("vcf_cbaac_tiled_prior", k.ptr, n, pr.ptr, hist.ptr, st.handle)
            L.call("vcf_cbaac_tiled_encode_prior", k.ptr, n, coder.order, pr.ptr, coder.seg_len, ob.ptr, cap,
                   sb.ptr, ws.ptr, st.handle)
        else:
            L.call("vcf_cbaac_tiled_encode", k.ptr, n, coder.order, coder.seg_len, ob.ptr, cap, sb.ptr, ws.ptr,
                   st.handle)
        st.synchronize()
        t4 = time.perf_counter()
        prior = None
        if coder.prior:
            prior = np.empty((K, 256) if K > 1 else 256, np.uint16)
            pr.download(prior, st)
        sizes = np.empty(ns + 1, np.int64)
        sb.download(sizes, st)
        st.synchronize()
        payload = np.empty(int(sizes[-1]), np.uint8)
        ob.download(payload, st)
        st.synchronize()
        t5 = time.perf_counter()
        import io
        cs = io.BytesIO(pack((Hp, Wp, 3), coder.order, coder.seg_len, sizes[:-1], payload.tobytes(), prior))
        with open(f"{out}_shape.bin", "wb") as f:
            f.write(struct.pack("iii", *img.shape))
        t6 = time.perf_counter()
        nbytes = c.encode_write_fn(cs, out)
        t7 = time.perf_counter()
        if it:
            for key, a, b in (("read", t0, t1), ("h2d", t1, t2), ("dct", t2, t3), ("entropy", t3, t4),
                              ("d2h", t4, t5), ("pack", t5, t6), ("write", t6, t7)):
                t[key].append((b - a) * 1e3)
    return {k: med(v) for k, v in t.items()}, nbytes


def stages_host_coder(c, src, out, reps):
    t = {k: [] for k in ("read", "h2d_dct_d2h", "entropy_host", "write")}
    for it in range(reps + 1):
        t0 = time.perf_counter()
        img = c.encode_read_fn(src)
        t1 = time.perf_counter()
        k = c.encode_indices(img)
        t2 = time.perf_counter()
        cs = c.compress(k)
        t3 = time.perf_counter()
        with open(f"{out}_shape.bin", "wb") as f:
            f.write(struct.pack("iii", *img.shape))
        nbytes = c.encode_write_fn(cs, out)
        t4 = time.perf_counter()
        if it:
            for key, a, b in (("read", t0, t1), ("h2d_dct_d2h", t1, t2), ("entropy_host", t2, t3), ("write", t3, t4)):
                t[key].append((b - a) * 1e3)
    return {k: med(v) for k, v in t.items()}, nbytes


def whole(c, src, out, reps):
    c.encode_fn(src, out)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        nbytes = c.encode_fn(src, out)
        ts.append((time.perf_counter() - t0) * 1e3)
    return med(ts), nbytes


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    set_device(0)
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "f.png")
        Image.fromarray(bench.synth_frame(1080, 1920, 0)).save(src)
        png_bytes = os.path.getsize(src)
        out = os.path.join(d, "e")
        for ec in ("TCBAAC", "TCBAACP", "CBAAC"):
            c = CoDec(P.parse(P.dct_parser(), ["encode", "-c", ec]))
            ms, nbytes = whole(c, src, out, reps)
            if ec == "CBAAC":
                st, nb2 = stages_host_coder(c, src, out, reps)
            else:
                st, nb2 = stages_gpu_coder(c, src, out, reps)
            assert nb2 == nbytes, (nb2, nbytes)
            print(json.dumps(dict(case="c2_encode_fn_stages", entropy=ec, frame=[1080, 1920, 3], png_bytes=png_bytes,
                                  encode_fn_ms=ms, stages_ms=st, stages_sum_ms=round(sum(st.values()), 3),
                                  bytes=nbytes, reps=reps)), flush=True)


if __name__ == "__main__":
    main()
