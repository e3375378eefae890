"""2D-DWT image codec: the drop-in for src/2D-DWT.py's CoDec.

Same constructor (argparse Namespace with levels, wavelet, color_transform,
quantizer, QSS, ...), same methods and files: encode_fn writes
{out}_LL_{L}.tif (uint16, LL + 128) and {out}_{LH,HL,HH}_{r}.tif (uint8,
+ 128) for r = L..1 and returns the bytes written (2D-DWT.py:57-78,
162-200); decode_fn reads them back and writes the decoded image
(:80-101, 202-228).  The span between the image and the subband arrays runs
on the GPU through libvcf_amd.so (vcf_dwt_dz_encode / vcf_dwt_dz_decode).
"""
from __future__ import annotations

import logging
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .. import dwt as DW
from .eic import CoDec as EICCoDec
from .tiff import TIFFCodec


class CoDec(EICCoDec):
    """2D-DWT.CoDec (2D-DWT.py:39-200) over YCoCg / deadzone / no_filter / TIFF."""

    def __init__(self, args):
        super().__init__(args)
        self.levels = int(getattr(args, "levels", 5))
        self.wavelet = str(getattr(args, "wavelet", "db5"))
        DW.wavelet_index(self.wavelet)            # ValueError for names pywt does not know
        ct = getattr(args, "color_transform", "YCoCg")
        # -t YCrCb only changes the base class: 2D-DWT.py binds from_RGB/to_RGB from
        # color_transforms.YCoCg at import (:19-20), so the arithmetic stays YCoCg's
        # (tests/golden/manifest_plugins.json "same_as_ycocg")
        if ct not in ("YCoCg", "YCrCb"):
            raise NotImplementedError(f"color transform {ct!r}: YCoCg (and YCrCb, which 2D-DWT.py runs as "
                                      "YCoCg) are on the HIP path")
        quant = getattr(args, "quantizer", "deadzone")
        if quant != "deadzone":
            raise NotImplementedError(f"quantizer {quant!r}: only deadzone is on the HIP path")
        filt = getattr(args, "filter", "no_filter")
        if not self.encoding and filt != "no_filter":
            raise NotImplementedError(f"filter {filt!r}: only no_filter is on the HIP path")
        ec = getattr(args, "entropy_image_codec", "TIFF")
        if ec != "TIFF":
            raise NotImplementedError(f"entropy codec {ec!r}: the DWT path writes TIFF subbands")
        self.entropy = TIFFCodec()
        self.file_extension = self.entropy.file_extension
        self.QSS = int(getattr(args, "QSS", 32))
        # opt-in (no reference counterpart): the lifting form of bior4.4, within
        # +-1 of the bit-exact path (the lifting form); args.dwt_lifting or VCF_DWT_LIFTING=1
        self.lifting = bool(getattr(args, "dwt_lifting", False)) or os.environ.get("VCF_DWT_LIFTING") == "1"
        if self.lifting:
            logging.warning("2D-DWT: the opt-in lifting path is selected (%s): indices and decoded bytes are "
                            "within +-1 of the reference, not bit-exact",
                            "args.dwt_lifting" if getattr(args, "dwt_lifting", False) else "VCF_DWT_LIFTING=1")
        if self.lifting and self.wavelet != "bior4.4":
            raise NotImplementedError("the lifting path is bior4.4 (CDF 9/7) only")
        logging.info(f"levels = {self.levels}")
        logging.info(f"wavelet={self.wavelet}")

    def compress(self, img):
        return self.entropy.compress(img)

    def decompress(self, codestream):
        return self.entropy.decompress(codestream)

    # ---- subband files (2D-DWT.py:162-228) ----------------------------------
    def write_decom_fn(self, subbands, fn):
        """subbands: {name: u16 LL / u8 detail array}, already + 128."""
        size = 0
        for name in DW.subband_names(self.levels):
            size += self.encode_write_fn(self.compress(subbands[name]), f"{fn}_{name}")
        return size

    def read_decom_fn(self, fn):
        return {name: self.decompress(self.decode_read_fn(f"{fn}_{name}")) for name in DW.subband_names(self.levels)}

    # ---- the hot path ---------------------------------------------------------
    def encode_fn(self, in_fn, out_fn):
        img = self.encode_read_fn(in_fn)
        if img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
            raise ValueError("Input image must be a 3D array (height, width, channels).")
        subbands = DW.encode(img, self.wavelet, self.levels, self.QSS, lifting=self.lifting)[0]
        return self.write_decom_fn(subbands, out_fn)

    def encode(self):
        # 2D-DWT.py:103-106: uses -o / -e
        return self.encode_fn(in_fn=self.args.original, out_fn=self.args.encoded)

    def _geometry(self, subbands):
        """H, W whose 'per' pyramid has these subband shapes (the level-1
        shapes fix every coarser one: ceil halving)."""
        h1, w1 = subbands[f"HH_1"].shape[:2]
        shapes, _, _ = DW.layout(2 * h1, 2 * w1, self.levels)
        for r, (h, w) in enumerate(shapes, start=1):
            for s in ("LH", "HL", "HH"):
                if subbands[f"{s}_{r}"].shape[:2] != (h, w):
                    raise ValueError(f"subband {s}_{r} has shape {subbands[f'{s}_{r}'].shape}, expected {(h, w)}")
        if subbands[f"LL_{self.levels}"].shape[:2] != shapes[-1]:
            raise ValueError("LL subband shape does not match the detail subbands")
        return 2 * h1, 2 * w1

    def decode_fn(self, in_fn, out_fn):
        subbands = self.read_decom_fn(in_fn)
        H, W = self._geometry(subbands)
        y = DW.decode(subbands, H, W, self.wavelet, self.levels, self.QSS, lifting=self.lifting)
        size = self.decode_write_fn(y, out_fn)
        self.BPP = (self.total_input_size * 8) / (y.shape[0] * y.shape[1])
        return size

    def decode(self):
        return self.decode_fn(in_fn=self.args.encoded, out_fn=self.args.decoded)

    # ---- batched frames (III runner) --------------------------------------------
    def encode_fns(self, pairs, batch: int = 16, io_threads: int = 8):
        pairs = list(pairs)
        sizes = [0] * len(pairs)
        with ThreadPoolExecutor(max_workers=io_threads) as pool:
            for b0 in range(0, len(pairs), batch):
                chunk = pairs[b0:b0 + batch]
                imgs = list(pool.map(lambda p: self.encode_read_fn(p[0]), chunk))
                groups = {}
                for i, img in enumerate(imgs):
                    if img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
                        raise ValueError("Input image must be a 3D array (height, width, channels).")
                    groups.setdefault(img.shape, []).append(i)
                sbs = [None] * len(chunk)
                for shape, idx in groups.items():
                    for j, sb in zip(idx, DW.encode(np.stack([imgs[i] for i in idx]), self.wavelet, self.levels,
                                                    self.QSS, lifting=self.lifting)):
                        sbs[j] = sb
                for i, s in enumerate(pool.map(lambda i: self.write_decom_fn(sbs[i], chunk[i][1]), range(len(chunk)))):
                    sizes[b0 + i] = s
        return sizes

    def decode_fns(self, pairs, batch: int = 16, io_threads: int = 8):
        return [self.decode_fn(i, o) for i, o in pairs]

    # ---- quantizer surface on subband lists (2D-DWT.py:113-160) -------------------
    def quantize_decom_fn(self, decom, fn=None):
        from .. import quant
        return [quant.deadzone_quantize(decom[0], self.QSS)] + \
            [tuple(quant.deadzone_quantize(b, self.QSS) for b in r) for r in decom[1:]]

    def dequantize_decom_fn(self, decom_k, fn=None):
        from .. import quant
        return [quant.deadzone_dequantize(decom_k[0], self.QSS)] + \
            [tuple(quant.deadzone_dequantize(b, self.QSS) for b in r) for r in decom_k[1:]]
