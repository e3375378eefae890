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


class YCoCgCoDec(_PixelCoDec):
    """YCoCg.CoDec (src/YCoCg.py:23-85), the stand-alone colour codec and the
    reference's default -t, over -a deadzone (one fused kernel per direction)
    or -a LloydMax (the int16 YCoCg image through the quantizer plug-in)."""

    def __init__(self, args):
        super().__init__(args)
        self.lm = make_quantizer(args)
        # :27-30: residues centred at zero for deadzone, Y - 128 otherwise
        self.offset = np.array([0, 0, 0]) if self.lm is None else np.array([-128, 0, 0])

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
        """:33-56: int16, from_RGB, + offset, quantize, astype(uint16), compress, write."""
        img = self.encode_read_fn(in_fn)
        self._check(img)
        H, W = img.shape[:2]
        if self.lm is None:
            k = PL.ycocg_dz_encode(img, self.QSS)
        else:
            from .._lib import call
            src = DeviceBuffer.from_array(img)
            ycc = DeviceBuffer(max(H * W * 3 * 2, 1))
            call("vcf_ycocg_i16_from_rgb", src.ptr, H * W, int(self.offset[0]), ycc.ptr, None)
            src.free()
            # k = empty_like(int16) <- searchsorted indices (0..N-1), astype(uint16): the same values
            dk = self.lm.quantize_device(ycc, np.int16, H * W, 3, np.uint16)
            ycc.free()
            self._take_codebook()
            k = dk.download(np.empty((H, W, 3), np.uint16))
            dk.free()
        return self.encode_write_fn(self.compress(k), out_fn)

    def decode_fn(self, in_fn, out_fn):
        """:58-85: decompress, astype(int16), dequantize, - offset, to_RGB, clip, uint8, filter, write."""
        k = self.decompress(self.decode_read_fn(in_fn))
        if k.ndim != 3 or k.shape[2] != 3:
            raise ValueError(f"index array of shape {k.shape}: expected H x W x 3")
        H, W = k.shape[:2]
        if self.lm is None:
            y = PL.ycocg_dz_decode(np.ascontiguousarray(k, dtype=np.uint16), self.QSS)
        else:
            from .._lib import call
            # y = empty_like(k.astype(int16)) <- centroids truncated into int16
            dk = DeviceBuffer.from_array(np.ascontiguousarray(k.astype(np.int16)))
            yc = self.lm.dequantize_device(dk, np.int16, H * W, 3, np.int16)
            dk.free()
            rgb = DeviceBuffer(max(H * W * 3, 1))
            call("vcf_ycocg_i16_to_rgb", yc.ptr, H * W, int(self.offset[0]), rgb.ptr, None)
            yc.free()
            y = rgb.download(np.empty((H, W, 3), np.uint8))
            rgb.free()
        return self.decode_write_fn(self.filter(y), out_fn)


class DeadzoneCoDec(_PixelCoDec):
    """deadzone.CoDec (src/deadzone.py:39-117) run as its own codec: the image
    quantized directly (int16, (x / Q) truncated, uint8) and back (Q * k in
    uint8), elementwise on the GPU."""

    def __init__(self, args, min_index_val=0, max_index_val=255):
        super().__init__(args)
        self.lm = None
        self.min_index_val, self.max_index_val = min_index_val, max_index_val

    def quantize(self, img, fn="/tmp/encoded"):
        from .. import quant
        return quant.deadzone_quantize(img, self.QSS)

    def dequantize(self, k, fn="/tmp/encoded"):
        from .. import quant
        return quant.deadzone_dequantize(k, self.QSS)

    def encode_fn(self, in_fn, out_fn):
        """:67-79: astype(int16), quantize, astype(uint8), compress, write."""
        img = self.encode_read_fn(in_fn)
        if img.dtype != np.uint8:
            raise NotImplementedError(f"{img.dtype} images: the HIP path takes u8 images")
        k = PL.dz_u8_encode(img, self.QSS)
        return self.encode_write_fn(self.compress(k), out_fn)

    def decode_fn(self, in_fn, out_fn):
        """:81-93: decompress, dequantize (Q * k in uint8), filter, write."""
        k = self.decompress(self.decode_read_fn(in_fn))
        if k.dtype != np.uint8:
            raise NotImplementedError(f"{k.dtype} indices: deadzone.py writes uint8")
        if self.QSS > 255:
            raise NotImplementedError(f"QSS {self.QSS}: Q * k is uint8 only for Q <= 255 (numpy value-based "
                                      "casting); the HIP path covers that case")
        y = PL.dz_u8_decode(k, self.QSS)
        return self.decode_write_fn(self.filter(y), out_fn)


class EntropyImageCoDec(EICCoDec):
    """An entropy codec run on the image itself: TIFF.py, CBAAC.py and
    CBAHC.py as stand-alone codecs (entropy_image_coding.CoDec.encode/decode,
    :81-86 / :117-121: read, compress, write; read, decompress, write)."""

    codec_name = "TIFF"

    def __init__(self, args):
        super().__init__(args)
        from argparse import Namespace
        self.entropy = make_entropy(Namespace(**{**vars(args), "entropy_image_codec": self.codec_name}))
        self.file_extension = self.entropy.file_extension

    def compress(self, img, fn="/tmp/encoded"):
        if self.codec_name == "CBAHC":
            return self.entropy.compress(img, fn)
        return self.entropy.compress(img)

    def decompress(self, codestream, fn="/tmp/encoded"):
        if self.codec_name == "CBAHC":
            return self.entropy.decompress(codestream, fn)
        return self.entropy.decompress(codestream)

    def compress_fn(self, img, fn):
        return self.compress(img, fn)

    def decompress_fn(self, codestream, fn):
        return self.decompress(codestream, fn)

    def encode_fn(self, in_fn, out_fn):
        img = self.encode_read_fn(in_fn)
        return self.encode_write_fn(self.compress(img), out_fn)

    def decode_fn(self, in_fn, out_fn):
        img = self.decompress(self.decode_read_fn(in_fn))
        if self.codec_name == "CBAAC":
            img = np.asarray(img).astype(np.uint8)      # CBAAC.py:112
        return self.decode_write_fn(img, out_fn)

    def encode(self):
        return self.encode_fn("/tmp/original.png", "/tmp/encoded")

    def decode(self):
        return self.decode_fn("/tmp/encoded", "/tmp/decoded.png")


class TIFFImageCoDec(EntropyImageCoDec):
    """TIFF.CoDec (src/TIFF.py:16-39)."""
    codec_name = "TIFF"


class CBAACImageCoDec(EntropyImageCoDec):
    """CBAAC.CoDec (src/CBAAC.py:72-156) with --order (:158-166)."""
    codec_name = "CBAAC"


class CBAHCImageCoDec(EntropyImageCoDec):
    """CBAHC.CoDec (src/CBAHC.py:158-283) with --order (:14-16)."""
    codec_name = "CBAHC"
