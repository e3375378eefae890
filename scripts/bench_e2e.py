#!/usr/bin/env python3
"""End-to-end III encode (config C4 shape: 1080p frames, DCT+deadzone+TIFF):
PNG files in, .tif + _shape.bin files out, through vcf_amd.codec.iii on one
GPU.  One JSON line per run with the whole-job rate and a stage breakdown
measured separately (PNG decode alone, GPU encode incl. PCIe alone, TIFF
deflate + write alone), so the bound is visible.

    python scripts/bench_e2e.py [--frames 64] [--threads 16] [--batch 32]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from PIL import Image

import bench
from vcf_amd.codec import parser as P
from vcf_amd.codec.dct2d import CoDec
from vcf_amd.device import set_device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--W", type=int, default=1920)
    a = ap.parse_args()
    set_device(0)
    tmp = tempfile.mkdtemp(prefix="vcf_e2e_")
    try:
        base = [bench.synth_frame(a.H, a.W, s) for s in range(8)]
        src = [os.path.join(tmp, f"original_{i:04d}.png") for i in range(a.frames)]
        with ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(lambda i: Image.fromarray(np.roll(base[i % 8], i, 1)).save(src[i], compress_level=1),
                        range(a.frames)))
        pairs = [(s, os.path.join(tmp, f"encoded_{i:04d}")) for i, s in enumerate(src)]
        codec = CoDec(P.parse(P.dct_parser(), ["encode"]))
        codec.encode_fns(pairs[:a.batch], batch=a.batch, io_threads=a.threads)   # warm-up (library, pools)
        t0 = time.perf_counter()
        sizes = codec.encode_fns(pairs, batch=a.batch, io_threads=a.threads)
        t_e2e = time.perf_counter() - t0
        px = a.frames * a.H * a.W
        # stage breakdown, each stage alone
        t0 = time.perf_counter()
        with ThreadPoolExecutor(a.threads) as ex:
            imgs = list(ex.map(codec.encode_read_fn, src))
        t_read = time.perf_counter() - t0
        import vcf_amd.dct as D
        t0 = time.perf_counter()
        ks = []
        for b0 in range(0, a.frames, a.batch):
            ks.extend(D.encode(np.stack(imgs[b0:b0 + a.batch]), 32, 0))
        t_gpu = time.perf_counter() - t0
        t0 = time.perf_counter()
        with ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(lambda i: codec.encode_write_fn(codec.compress(ks[i]), pairs[i][1] + "_w"), range(a.frames)))
        t_write = time.perf_counter() - t0
        # decode side: .tif + _shape.bin -> decoded PNG files
        dpairs = [(p[1], os.path.join(tmp, f"decoded_{i:04d}.png")) for i, p in enumerate(pairs)]
        dcodec = CoDec(P.parse(P.dct_parser(), ["decode"]))
        dcodec.decode_fns(dpairs[:a.batch], batch=a.batch, io_threads=a.threads)
        t0 = time.perf_counter()
        dcodec.decode_fns(dpairs, batch=a.batch, io_threads=a.threads)
        t_dec = time.perf_counter() - t0
        # the same with the strips inflated on host threads (round 3's path)
        from vcf_amd.codec.tiff import TIFFCodec
        TIFFCodec.gpu_batches = False
        t0 = time.perf_counter()
        dcodec.decode_fns(dpairs, batch=a.batch, io_threads=a.threads)
        t_dec_host = time.perf_counter() - t0
        TIFFCodec.gpu_batches = True
        print(json.dumps({
            "metric": "Mpixels/s III decode end to end (.tif files -> PNG files), 1 GPU",
            "value": round(px / t_dec / 1e6, 1), "unit": "Mpixels/s", "frames": a.frames,
            "frame": [a.H, a.W, 3], "threads": a.threads, "batch": a.batch,
            "tiff_inflate": "GPU (vcf_inflate_strips)",
            "host_inflate_value": round(px / t_dec_host / 1e6, 1)}), flush=True)
        print(json.dumps({
            "metric": "Mpixels/s III encode end to end (PNG files -> .tif files), 1 GPU",
            "value": round(px / t_e2e / 1e6, 1), "unit": "Mpixels/s", "frames": a.frames,
            "frame": [a.H, a.W, 3], "threads": a.threads, "batch": a.batch,
            "bytes_out": int(sum(sizes)),
            "stage_alone_Mpix_s": {"png_decode": round(px / t_read / 1e6, 1),
                                   "gpu_encode_incl_pcie": round(px / t_gpu / 1e6, 1),
                                   "tiff_deflate_write": round(px / t_write / 1e6, 1)},
            "host_cpus": os.cpu_count()}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
