"""TIFF strip deflate (TIFF.py:29: tifffile -> zlib level 6 per ~64 KB strip):
GPU vcf_zlib_strips vs the host path (system zlib on a thread pool), on the
index frames the DCT encode leaves in HBM (1080p and 4K, S-smooth content, Q=32)
and on raw RGB frames.  Every GPU strip is checked against zlib.compress.
Prints one JSON line per workload."""
import argparse
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--only", default="", help="comma-separated workload names")
    args = ap.parse_args()
    from vcf_amd.synthetic import synth_frame
    from vcf_amd import _lib as L
    from vcf_amd import dct
    from vcf_amd.codec.tiff import strip_layout
    from vcf_amd.device import DeviceBuffer, Event, Stream
    st = Stream()
    from vcf_amd.synthetic import c4_frame
    sets = [("dct_1080p", (1080, 1920), "dct"), ("dct_c4_1080p", (1080, 1920), "c4"), ("dct_4k", (2160, 3840), "dct"),
            ("rgb_1080p", (1080, 1920), "rgb")]
    if args.only:
        sets = [t for t in sets if t[0] in args.only.split(",")]
    for name, (H, W), kind in sets:
        n = args.frames if H == 1080 else max(1, args.frames // 4)
        if kind == "c4":   # bench.py's C4 sequence (shifted S-smooth frames, u8 wrap)
            bases = [synth_frame(H, W, seed=100 + s) for s in range(4)]
            frames = np.stack([c4_frame(bases, i) for i in range(n)])
            kind = "dct"
        else:
            base = np.stack([synth_frame(H, W, s) for s in range(4)])
            frames = base[np.arange(n) % 4]
        if kind == "dct":
            frames = np.concatenate([dct.encode(frames[i:i + 16], Q=32) for i in range(0, n, 16)])
        flat = np.ascontiguousarray(frames.reshape(n, -1))
        fb = flat.shape[1]
        _, _, sb = strip_layout(frames.shape[1:], 1)
        spf = int(L.lib().vcf_zlib_strip_count(fb, sb))
        total = spf * n
        slot = int(L.lib().vcf_zlib_bound(sb))
        d = DeviceBuffer.from_array(flat)
        out = DeviceBuffer(total * slot)
        sizes = DeviceBuffer(total * 4)
        ws = DeviceBuffer(int(L.lib().vcf_zlib_workspace(total)))
        e0, e1 = Event(), Event()
        ms = []
        for r in range(args.reps + 1):
            e0.record(st)
            L.call("vcf_zlib_strips", d.ptr, n, fb, sb, 6, out.ptr, slot, sizes.ptr, ws.ptr, st.handle)
            e1.record(st)
            st.synchronize()
            if r:
                ms.append(e0.elapsed_ms(e1))
            print(f"{name} rep {r}: {e0.elapsed_ms(e1):.2f} ms", file=sys.stderr, flush=True)
        sz = sizes.download(np.empty(total, np.int32))
        slots = out.download(np.empty(total * slot, np.uint8))
        # check every strip of frames 0 and n-1, and a sample elsewhere
        chk = sorted(set(list(range(spf)) + list(range((n - 1) * spf, total)) + list(range(0, total, 37))))
        bad = [s for s in chk if slots[s * slot:s * slot + sz[s]].tobytes() !=
               zlib.compress(flat[s // spf, (s % spf) * sb:(s % spf + 1) * sb].tobytes(), 6)]
        ok = not bad
        if bad:
            print(f"{name}: {len(bad)} of {len(chk)} checked strips differ from zlib, first {bad[:12]}",
                  file=sys.stderr, flush=True)
        # host: zlib on a thread pool over the same strips
        strips = [flat[f, k * sb:(k + 1) * sb] for f in range(n) for k in range(spf)]
        with ThreadPoolExecutor(args.threads) as ex:
            t = time.perf_counter()
            comp = list(ex.map(lambda c: zlib.compress(c, 6), strips))
            host_s = time.perf_counter() - t
        gms = float(np.median(ms))
        # the decode side: the GPU's own streams inflated on the GPU (vcf_inflate_strips),
        # straight from their slots into a frame buffer, against zlib.decompress on the pool
        k_of = np.arange(total) % spf
        out_len = np.minimum(sb, fb - k_of * sb).astype(np.int32)
        out_off = ((np.arange(total) // spf) * fb + k_of * sb).astype(np.int64)
        comp_off = (np.arange(total, dtype=np.int64) * slot)
        dco, dcl = DeviceBuffer.from_array(comp_off), DeviceBuffer.from_array(sz.astype(np.int32))
        doo, dol = DeviceBuffer.from_array(out_off), DeviceBuffer.from_array(out_len)
        dst, dimg = DeviceBuffer(4 * total), DeviceBuffer(flat.nbytes)
        ims = []
        for r in range(args.reps + 1):
            e0.record(st)
            L.call("vcf_inflate_strips", out.ptr, dco.ptr, dcl.ptr, total, dimg.ptr, doo.ptr, dol.ptr, dst.ptr,
                   st.handle)
            e1.record(st)
            st.synchronize()
            if r:
                ims.append(e0.elapsed_ms(e1))
        status = dst.download(np.empty(total, np.int32))
        inflate_ok = bool((status == 0).all() and np.array_equal(dimg.download(np.empty_like(flat)), flat))
        comp_strips = [slots[s * slot:s * slot + sz[s]].tobytes() for s in range(total)]
        with ThreadPoolExecutor(args.threads) as ex:
            t = time.perf_counter()
            list(ex.map(zlib.decompress, comp_strips))
            host_inf_s = time.perf_counter() - t
        ims_med = float(np.median(ims))
        for b in (dco, dcl, doo, dol, dst, dimg):
            b.free()
        print(json.dumps({"workload": f"{name}: {n} frames, {total} strips of {sb} B, zlib level 6",
                          "gpu_ms": round(gms, 3), "gpu_GBps": round(flat.nbytes / gms / 1e6, 2),
                          "host_ms": round(host_s * 1e3, 2), "host_threads": args.threads,
                          "host_GBps": round(flat.nbytes / host_s / 1e9, 3),
                          "speedup": round(host_s * 1e3 / gms, 2),
                          "ratio": round(flat.nbytes / max(1, int(sz.sum())), 2),
                          "bytes_equal_zlib": bool(ok and sum(map(len, comp)) == int(sz.sum())),
                          "strips_checked": len(chk),
                          "inflate_gpu_ms": round(ims_med, 3), "inflate_gpu_GBps": round(flat.nbytes / ims_med / 1e6, 2),
                          "inflate_host_ms": round(host_inf_s * 1e3, 2),
                          "inflate_equal_input": inflate_ok}), flush=True)
        for b in (d, out, sizes, ws):
            b.free()


if __name__ == "__main__":
    main()
