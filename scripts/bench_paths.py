#!/usr/bin/env python3
"""Secondary measurements (one JSON line each), beside bench.py's headline:

  dwt_encode / dwt_decode  4K 2D-DWT l=5 bior4.4 + deadzone (config C3), frames resident in HBM
  dct_decode               4K DCT+deadzone decode (64 frames resident)
  dct_encode_pcie          4K encode incl. host->device and device->host copies (pinned buffers)
  cbaac / cbahc            host entropy coders on a 1080p k-array (config C2), symbols/s
  configs                  whole-codec runs of configs C2 (CBAAC) and C5 (IPP) with files

Usage: python scripts/bench_paths.py [--only name,name]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
import vcf_amd._lib as L
from vcf_amd.device import DeviceBuffer, Event, Stream, set_device

HBM = 8000.0


def timed(stream, fn, steps, warmup, settle_s=0.5):
    """ms per call over `steps` calls, after `warmup` calls and at least
    settle_s seconds of back-to-back launches (the clocks ramp over the first
    ~30 launches)."""
    t0 = time.perf_counter()
    n = 0
    while n < warmup or time.perf_counter() - t0 < settle_s:
        fn()
        n += 1
        if n % 8 == 0:
            stream.synchronize()
    stream.synchronize()
    e0, e1 = Event(), Event()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    stream.synchronize()
    return e0.elapsed_ms(e1) / steps


def cpu_port(fn, px, what, budget=3.0):
    """The oracle (test infrastructure: the checker) timed on this host, 1 thread,
    for ~budget seconds, as the cpu_baseline beside a GPU line; returns it and
    the last output (compared with the GPU's by the caller)."""
    n, t0 = 0, time.perf_counter()
    while True:
        out = fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget:
            break
    return dict(value=round(n * px / el / 1e6, 3), unit="Mpixels/s", cores=1, kind="port",
                sample=f"{n} x {what}, {el:.1f} s"), out


def dwt(args):
    import vcf_amd.dwt as DW
    H, W, F, L_, Q = 2160, 3840, 8, 5, 32
    w = DW.wavelet_index("bior4.4")
    shapes, pb, wb = DW.layout(H, W, L_)
    frames = np.stack([bench.synth_frame(H, W, s) for s in range(F)])
    din, dpk, dws = DeviceBuffer.from_array(frames), DeviceBuffer(F * pb), DeviceBuffer(F * wb)
    Ho, Wo = 2 * shapes[0][0], 2 * shapes[0][1]
    dout = DeviceBuffer(F * Ho * Wo * 3)
    s = Stream()
    px = F * H * W
    from oracle import oracle as O
    cpu_e, sb = cpu_port(lambda: O.dwt_encode_frame(frames[0], "bior4.4", L_, Q), H * W,
                         "one 4K S-smooth frame, oracle/vcf_dwt_oracle.cpp (pywt 1.1.1 'per' restated)")
    cpu_d, _ = cpu_port(lambda: O.dwt_decode_frame(sb, H, W, "bior4.4", L_, Q), H * W,
                        "one 4K frame's subbands, oracle/vcf_dwt_oracle.cpp")
    names = {0: "default (two-chunk frame pipeline; fused level 1, strips for the middle levels, "
                "separable last level)",
             1: "fused level kernels", 2: "separable kernels"}
    for variant in [int(v) for v in args.dwt_variants.split(",")]:
        vname = names.get(variant, f"variant {variant}")
        enc = lambda: L.dwt_encode_v(variant, din.ptr, F, H, W, w, L_, Q, dpk.ptr, dws.ptr,
                             s.handle)
        dec = lambda: L.dwt_decode_v(variant, dpk.ptr, F, H, W, w, L_, Q, dout.ptr, dws.ptr,
                             s.handle)
        te = timed(s, enc, args.steps, 2)
        td = timed(s, dec, args.steps, 2)
        for name, t, alg in (("dwt_encode", te, F * (H * W * 3 + pb)), ("dwt_decode", td, F * (pb + Ho * Wo * 3))):
            print(json.dumps({"metric": f"Mpixels/s {name} 4K l=5 bior4.4 Q=32", "variant": vname,
                              "value": round(px / t / 1e3, 1), "unit": "Mpixels/s", "ms_per_launch": round(t, 3),
                              "frames_per_launch": F, "alg_GBps": round(alg / t / 1e6, 1),
                              "frac_hbm_alg": round(alg / t / 1e6 / HBM, 4),
                              "cpu_baseline": cpu_e if name == "dwt_encode" else cpu_d}), flush=True)


def dct_decode(args):
    import vcf_amd.dct as D
    H, W, F, Q = 2160, 3840, 64, 32
    Hp, Wp = D.padded_shape(H, W)
    frames = [bench.synth_frame(H, W, s) for s in range(4)]
    din = DeviceBuffer(F * H * W * 3)
    for f in range(F):
        din.upload(frames[f % 4], offset=f * H * W * 3)
    dk, dout = DeviceBuffer(F * Hp * Wp * 3), DeviceBuffer(F * H * W * 3)
    s = Stream()
    D.encode_device(din, F, H, W, Q, out=dk, stream=s)
    alg = F * (Hp * Wp * 3 + H * W * 3)
    from oracle import oracle as O
    k0 = O.encode_frame(frames[0], Q)
    cpu, _ = cpu_port(lambda: O.decode_frame(k0, H, W, Q), H * W, "one 4K frame, oracle/vcf_oracle.c")
    for variant, vname in ((0, "default (column-per-lane, dequantization table, packed int16 epilogue)"),
                           (2, "column-per-lane, round-1 form"), (1, "lane-per-block")):
        t = timed(s, lambda: D.decode_device(dk, F, H, W, Q, out=dout, stream=s, variant=variant), args.steps, 3)
        print(json.dumps({"metric": "Mpixels/s dct_decode 4K Q=32", "variant": vname,
                          "value": round(F * H * W / t / 1e3, 1),
                          "unit": "Mpixels/s", "ms_per_launch": round(t, 4), "frames_per_launch": F,
                          "alg_GBps": round(alg / t / 1e6, 1), "frac_hbm": round(alg / t / 1e6 / HBM, 4),
                          "cpu_baseline": cpu}),
              flush=True)


def dct_encode_pcie(args):
    """Host frames in pinned memory -> HBM -> encode -> host, one stream, F frames per step."""
    import vcf_amd.dct as D
    H, W, F, Q = 2160, 3840, 16, 32
    Hp, Wp = D.padded_shape(H, W)
    nin, nout = F * H * W * 3, F * Hp * Wp * 3
    hin, hout = ctypes.c_void_p(), ctypes.c_void_p()
    L.call("vcf_host_alloc", ctypes.byref(hin), nin)
    L.call("vcf_host_alloc", ctypes.byref(hout), nout)
    src = np.ctypeslib.as_array((ctypes.c_uint8 * nin).from_address(hin.value))
    src[:] = np.tile(bench.synth_frame(H, W, 0).ravel(), F)
    din, dout = DeviceBuffer(nin), DeviceBuffer(nout)
    s = Stream()

    def step():
        L.call("vcf_memcpy_htod", din.ptr, hin, nin, s.handle)
        D.encode_device(din, F, H, W, Q, out=dout, stream=s)
        L.call("vcf_memcpy_dtoh", hout, dout.ptr, nout, s.handle)

    t = timed(s, step, args.steps, 2)
    print(json.dumps({"metric": "Mpixels/s dct_encode 4K incl. H2D+D2H (pinned, one stream)",
                      "value": round(F * H * W / t / 1e3, 1), "unit": "Mpixels/s", "ms_per_step": round(t, 3),
                      "frames_per_step": F, "pcie_GBps": round((nin + nout) / t / 1e6, 1)}), flush=True)
    L.call("vcf_host_free", hin)
    L.call("vcf_host_free", hout)


def ipp(args):
    """Config C5's temporal tools at 4K on resident frames: luma + block matching
    (16x16, S=8, full search and TSS) + compensation + residual, per P-frame."""
    H, W, bs, sr = 2160, 3840, 16, 8
    f0 = bench.synth_frame(H, W, 0)
    f1 = np.roll(f0, (3, 1), axis=(0, 1))          # S-motion: (3, 1) px per frame
    dr, dc = DeviceBuffer.from_array(f0), DeviceBuffer.from_array(f1)
    dmv, dg = DeviceBuffer((H // bs) * (W // bs) * 8), DeviceBuffer(2 * H * W)
    dcomp, dres = DeviceBuffer(H * W * 3), DeviceBuffer(H * W * 3)
    s = Stream()
    from oracle import oracle as O
    cpu = {fast: cpu_port(lambda: O.ipp_block_matching(f0, f1, bs, sr, bool(fast)), H * W,
                          "one 4K frame pair, oracle/vcf_ipp_oracle.c")[0] for fast in (0, 1)}
    for fast, kv in ((0, 0), (0, 1), (1, 0), (1, 1)):
        L.call("vcf_ipp_set_full_search_variant", kv)

        def me():
            L.call("vcf_ipp_block_match", dr.ptr, dc.ptr, H, W, bs, sr, fast, dmv.ptr, dg.ptr, s.handle)

        def pframe():
            me()
            L.call("vcf_ipp_motion_compensate", dr.ptr, dmv.ptr, H, W, bs, dcomp.ptr, s.handle)
            L.call("vcf_ipp_residual", dc.ptr, dcomp.ptr, H * W * 3, dres.ptr, s.handle)
        t_me = timed(s, me, args.steps, 3)
        t_p = timed(s, pframe, args.steps, 3)
        sads = (H // bs) * (W // bs) * (2 * sr + 1) ** 2 * bs * bs
        L.call("vcf_ipp_set_full_search_variant", 0)
        print(json.dumps({"metric": f"ipp {'tss' if fast else 'full-search'} motion estimation 4K bs=16 S=8",
                          "variant": ("three-step, " + ("serial kernel" if kv else "parallel rounds")) if fast
                          else ("byte kernel" if kv else "word kernel"),
                          "value": round(H * W / t_me / 1e3, 1), "unit": "Mpixels/s", "ms_per_frame": round(t_me, 4),
                          "p_frame_tools_ms": round(t_p, 4),
                          "note": ("289 candidates x 256 |diff| per block = %.2f G abs-diffs/frame" % (sads / 1e9))
                          if not fast else "serial three-step search, one wave per block",
                          "cpu_baseline": cpu[fast]}), flush=True)


def entropy(args):
    from vcf_amd import cbaac, cbahc
    import vcf_amd.dct as D
    rgb = bench.synth_frame(1080, 1920, 3)
    k = D.encode(rgb, 32)          # the 1080p index array config C2 entropy-codes
    sym = k.ravel()
    for name, mod in (("cbaac", cbaac), ("cbahc", cbahc)):
        for order in (0, 1):
            n = sym.size if name == "cbaac" else min(sym.size, 1 << 20)
            t0 = time.perf_counter()
            out = mod.encode_symbols(sym[:n], order)
            t1 = time.perf_counter()
            nbytes = len(out) if isinstance(out, bytes) else len(out[0])
            print(json.dumps({"metric": f"{name} order {order} encode (host, 1 thread)",
                              "value": round(n / (t1 - t0) / 1e6, 2), "unit": "Msymbols/s",
                              "symbols": n, "bits_per_symbol": round(8 * nbytes / n, 4),
                              "sample": "1080p S-smooth frame, DCT+deadzone indices (config C2)"}), flush=True)


def configs(args):
    """Whole-codec runs of BASELINE.json configs C2 and C5 on one GPU, files included.

    C2: 1080p frame -> 2D-DCT CoDec with -c CBAAC (encode_fn: PNG read, GPU
        transform + quantizer, host CBAAC order 0, file write), frames/s over
        16 frames coded by a 16-thread pool (frames are independent);
    C5: IPP_DCT CoDec over 4K frames from an .npy (I + P frames, GOP 10, full
        search bs 16 S 8: GPU ME/MC/residual/transform, host TIFF deflate, the
        reference's original-frame PNG dumps), frames/s."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    from vcf_amd.codec.ipp import CoDec as IPPCoDec
    tmp = tempfile.mkdtemp(prefix="vcf_cfg_")
    try:
        # C2
        n = 16
        srcs = []
        for i in range(n):
            srcs.append(os.path.join(tmp, f"c2_{i}.png"))
            Image.fromarray(bench.synth_frame(1080, 1920, i)).save(srcs[-1], compress_level=1)
        codec = CoDec(P.parse(P.dct_parser(), ["encode", "-c", "CBAAC"]))
        codec.encode_fn(srcs[0], os.path.join(tmp, "warm"))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(16) as ex:
            sizes = list(ex.map(lambda i: codec.encode_fn(srcs[i], os.path.join(tmp, f"c2_enc_{i}")), range(n)))
        t = time.perf_counter() - t0
        print(json.dumps({"metric": "config C2: 1080p 2D-DCT + deadzone + CBAAC encode_fn, files included",
                          "value": round(n * 1080 * 1920 / t / 1e6, 1), "unit": "Mpixels/s",
                          "frames_per_s": round(n / t, 2), "threads": 16, "frames": n,
                          "bits_per_pixel": round(8 * sum(sizes) / (n * 1080 * 1920), 4)}), flush=True)
        # C5
        nf = int(os.environ.get("C5_FRAMES", "20"))
        f0 = bench.synth_frame(2160, 3840, 0)
        frames = np.stack([np.roll(f0, (3 * t, t), axis=(0, 1)) for t in range(nf)])
        np.save(os.path.join(tmp, "c5.npy"), frames)
        argv = ["encode", "-i", os.path.join(tmp, "c5.npy"), "-O", os.path.join(tmp, "c5", "v"), "-N", str(nf),
                "-G", "10", "-M", "16", "-S", "8"]
        t0 = time.perf_counter()
        IPPCoDec(P.parse(P.ipp_parser(), argv)).encode()
        t = time.perf_counter() - t0
        print(json.dumps({"metric": "config C5: IPP_DCT encode of 4K frames (GOP 10, ME bs 16 S 8), files included",
                          "value": round(nf * 2160 * 3840 / t / 1e6, 1), "unit": "Mpixels/s",
                          "frames_per_s": round(nf / t, 2), "frames": nf,
                          "note": "serial within a GOP; includes the reference's PNG dumps of the originals"}),
              flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--only", default="dwt,dct_decode,dct_encode_pcie,ipp,entropy,configs")
    ap.add_argument("--dwt-variants", default="0,1,2")
    args = ap.parse_args()
    set_device(0)
    for name in args.only.split(","):
        globals()[name](args)


if __name__ == "__main__":
    main()
