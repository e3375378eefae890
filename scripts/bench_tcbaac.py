#!/usr/bin/env python3
"""Tiled CBAAC (§8(f) row 2) measurements on one GPU; one JSON line per case.

- rate: bits of the tiled stream vs the serial stream (vcf_cbaac_encode over
  the whole frame, the reference's CBAAC.py layout) for several segment
  lengths, on the indices of S-smooth 1080p / 4K frames (DCT B=8, Q=32);
- GPU time per frame (HIP events around the encode / decode launches, data
  resident in HBM) and the host serial coder's time for the same frame;
- C2 end to end: encode_fn of a 1080p PNG with -c TCBAAC (PNG read, DCT +
  tiled CBAAC on the GPU, file write) vs -c CBAAC (host coder), wall clock.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def frame_indices(H, W, seed=0, Q=32):
    from vcf_amd.synthetic import synth_frame
    import vcf_amd.dct as D
    return D.encode(synth_frame(H, W, seed), Q)


def time_gpu(fn, stream, reps):
    from vcf_amd.device import Event
    fn()
    stream.synchronize()
    e0, e1 = Event(), Event()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    stream.synchronize()
    return e0.elapsed_ms(e1) / reps


def case(H, W, order, seg_len, reps=5):
    from vcf_amd import _lib as L
    from vcf_amd import cbaac, tcbaac
    from vcf_amd.device import DeviceBuffer
    k = frame_indices(H, W)
    n = k.size
    coder = tcbaac.TiledCoder(order, seg_len)
    sizes, payload = coder.encode(k)
    # kernel timing: encode (code + scan + pack) with the symbols in HBM
    lib = L.lib()
    sym = DeviceBuffer.from_array(k.ravel(), coder.stream)
    ws = DeviceBuffer(int(lib.vcf_cbaac_tiled_workspace(n, seg_len)))
    cap = int(lib.vcf_cbaac_tiled_bound(n, seg_len))
    out = DeviceBuffer(cap)
    sb = DeviceBuffer(8 * (len(sizes) + 1))
    enc_ms = time_gpu(lambda: L.call("vcf_cbaac_tiled_encode", sym.ptr, n, order, seg_len, out.ptr, cap, sb.ptr,
                                     ws.ptr, coder.stream.handle), coder.stream, reps)
    dec_out = DeviceBuffer(n)
    coder.decode_to_device(payload, sizes, n, dec_out)
    offs = DeviceBuffer.from_array(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64), coder.stream)
    src = DeviceBuffer.from_array(np.frombuffer(payload, np.uint8), coder.stream)
    dec_ms = time_gpu(lambda: L.call("vcf_cbaac_tiled_decode", src.ptr, offs.ptr, n, order, seg_len, dec_out.ptr,
                                     coder.stream.handle), coder.stream, reps)
    back = np.empty(n, np.uint8)
    dec_out.download(back)
    t0 = time.perf_counter()
    serial = cbaac.encode_symbols(k, order)
    host_ms = (time.perf_counter() - t0) * 1e3
    return dict(case="tcbaac", frame=[H, W, 3], order=order, seg_len=seg_len, segments=len(sizes), symbols=n,
                serial_bytes=len(serial), tiled_bytes=len(payload),
                rate_overhead=round(len(payload) / len(serial) - 1, 4),
                bits_per_symbol=round(8 * len(payload) / n, 4),
                gpu_encode_ms=round(enc_ms, 3), gpu_decode_ms=round(dec_ms, 3),
                gpu_encode_Msym_s=round(n / enc_ms / 1e3, 1), gpu_decode_Msym_s=round(n / dec_ms / 1e3, 1),
                host_serial_ms=round(host_ms, 2), round_trip=bool(np.array_equal(back, k.ravel())))


def case_prior(H, W, seg_len, order=0, reps=5):
    """Container version 2 (order 0, models seeded by the frame's prior):
    rate vs the serial stream and GPU time per frame (prior + encode)."""
    from vcf_amd import _lib as L
    from vcf_amd import cbaac, tcbaac
    from vcf_amd.device import DeviceBuffer
    k = frame_indices(H, W)
    n = k.size
    coder = tcbaac.TiledCoder(order, seg_len, prior=True)
    sizes, payload = coder.encode(k)
    lib = L.lib()
    sym = DeviceBuffer.from_array(k.ravel(), coder.stream)
    ws = DeviceBuffer(int(lib.vcf_cbaac_tiled_workspace(n, seg_len)))
    cap = int(lib.vcf_cbaac_tiled_bound(n, seg_len))
    out, sb = DeviceBuffer(cap), DeviceBuffer(8 * (len(sizes) + 1))
    pr, hist = DeviceBuffer(512), DeviceBuffer(1024)

    def enc():
        L.call("vcf_cbaac_tiled_prior", sym.ptr, n, pr.ptr, hist.ptr, coder.stream.handle)
        L.call("vcf_cbaac_tiled_encode_prior", sym.ptr, n, order, pr.ptr, seg_len, out.ptr, cap, sb.ptr, ws.ptr,
               coder.stream.handle)
    enc_ms = time_gpu(enc, coder.stream, reps)
    dec_out = DeviceBuffer(n)
    offs = DeviceBuffer.from_array(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64), coder.stream)
    src = DeviceBuffer.from_array(np.frombuffer(payload, np.uint8), coder.stream)
    prd = DeviceBuffer.from_array(coder.last_prior, coder.stream)
    dec_ms = time_gpu(lambda: L.call("vcf_cbaac_tiled_decode_prior", src.ptr, offs.ptr, n, order, prd.ptr, seg_len,
                                     dec_out.ptr, coder.stream.handle), coder.stream, reps)
    back = np.empty(n, np.uint8)
    dec_out.download(back)
    serial = cbaac.encode_symbols(k, order)
    total = len(payload) + 512   # the prior table travels in the container
    return dict(case="tcbaac_prior", frame=[H, W, 3], order=order, seg_len=seg_len, segments=len(sizes), symbols=n,
                serial_bytes=len(serial), tiled_bytes=total, rate_overhead=round(total / len(serial) - 1, 4),
                gpu_encode_ms=round(enc_ms, 3), gpu_decode_ms=round(dec_ms, 3),
                round_trip=bool(np.array_equal(back, k.ravel())))


def frames_throughput(H, W, n_frames=16, seg_len=1 << 15, streams=8, reps=3):
    """n_frames frames' indices resident in HBM, each its own prior-seeded
    tiled stream, coded concurrently on `streams` library streams."""
    from vcf_amd import tcbaac
    from vcf_amd.device import DeviceBuffer
    k = frame_indices(H, W).ravel()
    n = k.size
    buf = DeviceBuffer.from_array(np.tile(k, n_frames))
    tcbaac.encode_frames_device(buf, n_frames, n, 0, seg_len, prior=True, streams=streams)   # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        res = tcbaac.encode_frames_device(buf, n_frames, n, 0, seg_len, prior=True, streams=streams)
    ms = (time.perf_counter() - t0) / reps * 1e3
    return dict(case="tcbaac_prior_frames", frame=[H, W, 3], frames=n_frames, seg_len=seg_len, streams=streams,
                ms_per_batch=round(ms, 2), ms_per_frame=round(ms / n_frames, 3),
                Mpix_s=round(n_frames * H * W / ms / 1e3, 1), bytes_per_frame=len(res[0][1]) + 512)


def c2_end_to_end(reps=5):
    from PIL import Image

    from vcf_amd.synthetic import synth_frame
    from vcf_amd.codec import parser as P
    from vcf_amd.codec.dct2d import CoDec
    rows = []
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "f.png")
        Image.fromarray(synth_frame(1080, 1920, 0)).save(src)
        for ec in ("TCBAAC", "TCBAACP", "CBAAC"):
            c = CoDec(P.parse(P.dct_parser(), ["encode", "-c", ec]))
            c.encode_fn(src, os.path.join(d, "e"))        # warm (allocations, first launch)
            t0 = time.perf_counter()
            for _ in range(reps):
                nbytes = c.encode_fn(src, os.path.join(d, "e"))
            ms = (time.perf_counter() - t0) / reps * 1e3
            rows.append(dict(case="c2_encode_fn", entropy=ec, frame=[1080, 1920, 3], ms_per_frame=round(ms, 2),
                             Mpix_s=round(1080 * 1920 / ms / 1e3, 1), bytes=nbytes))
    return rows


def main():
    from vcf_amd.device import set_device
    set_device(0)
    if "--frames" in sys.argv:
        for H, W in ((1080, 1920), (2160, 3840)):
            for seg, st in ((1 << 15, 1), (1 << 15, 8), (1 << 14, 8)):
                print(json.dumps(frames_throughput(H, W, 16, seg, st)), flush=True)
        return
    if "--c2" in sys.argv:
        for r in c2_end_to_end():
            print(json.dumps(r), flush=True)
        return
    if "--prior" in sys.argv:
        orders = (1,) if "--order1" in sys.argv else (0,) if "--order0" in sys.argv else (0, 1)
        for order in orders:
            for H, W in ((1080, 1920), (2160, 3840)):
                for seg in (1 << 12, 1 << 13, 1 << 14, 1 << 15, 1 << 17):
                    print(json.dumps(case_prior(H, W, seg, order)), flush=True)
        return
    for H, W in ((1080, 1920), (2160, 3840)):
        for order in (0, 1):
            for seg in (1 << 15, 1 << 16, 1 << 17, 1 << 18):
                print(json.dumps(case(H, W, order, seg)), flush=True)
    for r in c2_end_to_end():
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
