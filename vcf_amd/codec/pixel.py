"""The stand-alone pixel-domain codecs of §8(f) row 4, drop-ins for
src/LloydMax.py's and src/YCrCb.py's CoDec classes.

Both keep the reference's surface: CoDec(args), encode()/decode() with the
hard-wired default files of entropy_image_coding.py (encode() reads
/tmp/original.png and writes /tmp/encoded<ext>, decode() the reverse into
/tmp/decoded.png; -o/-e/-d are parsed but, as in the reference, not used by
these two methods), encode_fn/decode_fn taking explicit names, quantize /
dequantize, compress / decompress, bye().  The per-pixel span runs on the
GPU (vcf_amd.plugins): YCrCb + deadzone in one fused kernel per direction,
the colour transform and the LloydMax quantizer as separate kernels.
"""
from __future__ import annotations

import logging

import numpy as np

from .. import plugins as PL
from ..device import DeviceBuffer
from .dct2d import make_entropy, make_quantizer
from .eic import CoDec as EICCoDec
from .quantizers import LloydMaxQuantizer


class _PixelCoDec(EICCoDec):
    def __init__(self, args):
        super().__init__(args)
        filt = getattr(args, "filter", "no_filter")
        if not self.encoding and filt != "no_filter":
            raise NotImplementedError(f"filter {filt!r}: only no_filter is on the HIP path")
        self.entropy = make_entropy(args)
        self.file_extension = self.entropy.file_extension
        self.QSS = int(getattr(args, "QSS", 32))

    def compress(self, img):
        return self.entropy.compress(img)

    def decompress(self, codestream):
        return self.entropy.decompress(codestream)

    def filter(self, img):
        """no_filter.CoDec.filter (:31-34)."""
        return img

    def encode(self):
        return self.encode_fn("/tmp/original.png", "/tmp/encoded")

    def decode(self):
        return self.decode_fn("/tmp/encoded", "/tmp/decoded.png")

    def _check(self, img):
        if img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
            raise NotImplementedError(f"{img.dtype} {img.shape} images: the HIP path takes u8 RGB")

    def _take_codebook(self):
        if self.lm is not None:
            self.total_output_size += self.lm.codebook_bytes   # LloydMax.py:107-108
            self.lm.codebook_bytes = 0


class LloydMaxCoDec(_PixelCoDec):
    """LloydMax.CoDec (src/LloydMax.py:48-147): the image itself quantized per channel."""

    def __init__(self, args):
        super().__init__(args)
        self.min_val = int(getattr(args, "min_val", 0))
        self.max_val = int(getattr(args, "max_val", 255))
        self.lm = LloydMaxQuantizer(self.QSS, self.min_val, self.max_val)
        logging.info(f"min_val = {self.min_val}")
        logging.info(f"max_val = {self.max_val}")
        logging.info(f"QSS = {self.QSS}")

    def quantize(self, img, fn="/tmp/encoded"):
        return self.lm.quantize(img, fn)

    def dequantize(self, k, fn="/tmp/encoded"):
        return self.lm.dequantize(k, fn)

    def encode_fn(self, in_fn, out_fn):
        """:56-63: read, quantize (k = empty_like(img): uint8), compress, write."""
        img = self.encode_read_fn(in_fn)
        self._check(img)
        k = self.quantize(img)
        self._take_codebook()
        return self.encode_write_fn(self.compress(k), out_fn)

    def decode_fn(self, in_fn, out_fn):
        """:65-73: read, decompress, dequantize (y = empty_like(k): uint8), filter, write."""
        k = self.decompress(self.decode_read_fn(in_fn))
        y = self.dequantize(k)
        return self.decode_write_fn(self.filter(y), out_fn)


class YCrCbCoDec(_PixelCoDec):
    """YCrCb.CoDec (src/YCrCb.py:25-72) over -a deadzone (fused kernels) or -a LloydMax."""

    def __init__(self, args):
        super().__init__(args)
        self.lm = make_quantizer(args)
        self.offset = np.array([0, 0, 0])    # :27-31, both branches

    def quantize(self, img, fn="/tmp/encoded"):
        if self.lm is not None:
            return self.lm.quantize(img, fn)
        from .. import quant
        return quant.deadzone_quantize(img, self.QSS)

    def dequantize(self, k, fn="/tmp/encoded"):
        if self.lm is not None:
            return self.lm.dequantize(k, fn)
        from .. import quant
        return quant.deadzone_dequantize(k, self.QSS)

    def encode_fn(self, in_fn, out_fn):
        """:33-51: from_RGB, int16, + offset, quantize, uint16, compress, write."""
        img = self.encode_read_fn(in_fn)
        self._check(img)
        H, W = img.shape[:2]
        if self.lm is None:
            k = PL.ycrcb_dz_encode(img, self.QSS)
        else:
            # the int16 YCrCb values are the uint8 ones: the histogram, the thresholds and
            # k = empty_like(int16).astype(uint16) come out the same from the uint8 array
            src = DeviceBuffer.from_array(img)
            ycc = DeviceBuffer(img.nbytes)
            from .._lib import call
            call("vcf_ycrcb_from_rgb", src.ptr, H * W, ycc.ptr, None)
            src.free()
            dk = self.lm.quantize_device(ycc, np.uint8, H * W, 3, np.uint16)
            ycc.free()
            self._take_codebook()
            k = dk.download(np.empty((H, W, 3), np.uint16))
            dk.free()
        return self.encode_write_fn(self.compress(k), out_fn)

    def decode_fn(self, in_fn, out_fn):
        """:53-72: decompress, dequantize, int16, - offset, uint8, to_RGB, clip, filter, write."""
        k = self.decompress(self.decode_read_fn(in_fn))
        if k.ndim != 3 or k.shape[2] != 3:
            raise ValueError(f"index array of shape {k.shape}: expected H x W x 3")
        H, W = k.shape[:2]
        if self.lm is None:
            y = PL.ycrcb_dz_decode(np.ascontiguousarray(k, dtype=np.uint16), self.QSS)
        else:
            # y = empty_like(k) (uint16) <- centroids, astype(int16), astype(uint8): the low byte
            dk = DeviceBuffer.from_array(np.ascontiguousarray(k))
            yc = self.lm.dequantize_device(dk, k.dtype, H * W, 3, np.uint8)
            dk.free()
            rgb = DeviceBuffer(H * W * 3)
            from .._lib import call
            call("vcf_ycrcb_to_rgb", yc.ptr, H * W, rgb.ptr, None)
            yc.free()
            y = rgb.download(np.empty((H, W, 3), np.uint8))
            rgb.free()
        return self.decode_write_fn(self.filter(y), out_fn)
