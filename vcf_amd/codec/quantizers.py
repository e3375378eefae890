"""The LloydMax quantizer plug-in (src/LloydMax.py:75-147) over the GPU.

LloydMaxQuantizer mirrors LloydMax.CoDec's quantizer surface -- the side
files included: quantize_fn(img, fn) writes {fn}_params.txt (QSS, min_val,
max_val, one per line) and {fn}_centroids_<c>.gz (np.save of the float64
centroids inside a gzip stream, :85-107), and dequantize_fn(k, fn) reads
them back (:120-143).  As in the reference, the codecs call quantize(img) /
dequantize(k) with the hard-wired prefix /tmp/encoded (:112, :145), so the
side files always land there whatever -e says.  The per-sample work runs
in libvcf_amd.so (vcf_amd.plugins); k has img's dtype (k = empty_like(img),
:96) unless the caller asks for another, y has k's (:130).
"""
from __future__ import annotations

import gzip
import io
import logging
import os

import numpy as np

from .. import plugins as PL
from ..device import DeviceBuffer

DEFAULT_MIN_VAL = 0          # LloydMax.py:23
DEFAULT_MAX_VAL = 255        # :24
SIDE_PREFIX = "/tmp/encoded"


class LloydMaxQuantizer:
    def __init__(self, QSS: int, min_val: int = DEFAULT_MIN_VAL, max_val: int = DEFAULT_MAX_VAL):
        self.QSS, self.min_val, self.max_val = int(QSS), int(min_val), int(max_val)
        self.codebook_bytes = 0      # added to the codec's total_output_size (:107-108)

    # ---- side files ---------------------------------------------------------
    def write_side(self, fn: str, cents) -> int:
        with open(f"{fn}_params.txt", "w") as f:
            f.write(f"{self.QSS}\n{self.min_val}\n{self.max_val}\n")
        total = 0
        for c, cent in enumerate(cents):
            path = f"{fn}_centroids_{c}.gz"
            with gzip.GzipFile(path, "w") as f:
                np.save(file=f, arr=np.asarray(cent, np.float64))
            n = os.path.getsize(path)
            logging.info(f"Written {n} bytes in {path}")
            total += n
        self.codebook_bytes += total
        return total

    @staticmethod
    def read_side(fn: str, channels: int):
        with open(f"{fn}_params.txt", "r") as f:
            QSS, min_val, max_val = [int(line.strip()) for line in f]
        cents = []
        for c in range(channels):
            with gzip.GzipFile(f"{fn}_centroids_{c}.gz", "r") as f:
                cents.append(np.load(io.BytesIO(f.read()), allow_pickle=False))
        return (QSS, min_val, max_val), cents

    # ---- device arrays ------------------------------------------------------
    def quantize_device(self, x: DeviceBuffer, dtype, n_px: int, channels: int, k_dtype,
                        fn: str = SIDE_PREFIX, out: DeviceBuffer | None = None, stream=None) -> DeviceBuffer:
        k, cents = PL.lm_quantize_device(x, dtype, n_px, channels, self.QSS, self.min_val, self.max_val,
                                         k_dtype, out=out, stream=stream)
        self.write_side(fn, cents)
        return k

    def dequantize_device(self, k: DeviceBuffer, k_dtype, n_px: int, channels: int, y_dtype,
                          fn: str = SIDE_PREFIX, out: DeviceBuffer | None = None, stream=None) -> DeviceBuffer:
        _, cents = self.read_side(fn, channels)
        return PL.lm_dequantize_device(k, k_dtype, n_px, channels, cents, y_dtype, out=out, stream=stream)

    # ---- host arrays (the reference's quantize_fn / dequantize_fn) ----------
    def quantize_fn(self, img: np.ndarray, fn: str) -> np.ndarray:
        k, cents = PL.lm_quantize(img, self.QSS, self.min_val, self.max_val)
        self.write_side(fn, cents)
        return k

    def dequantize_fn(self, k: np.ndarray, fn: str) -> np.ndarray:
        C = k.shape[2] if k.ndim == 3 else 1
        _, cents = self.read_side(fn, C)
        return PL.lm_dequantize(k, cents)

    def quantize(self, img, fn=SIDE_PREFIX):
        return self.quantize_fn(img, fn)

    def dequantize(self, k, fn=SIDE_PREFIX):
        return self.dequantize_fn(k, fn)
