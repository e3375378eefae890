"""Shared I/O of the entropy image codecs: src/entropy_image_coding.py.

CoDec.encode_read_fn (:51-65) reads an image file into an H x W x 3 uint8
RGB array; encode_write_fn (:70-79) writes a code-stream as fn +
file_extension; decode_read_fn (:91-96) reads it back; decode_write_fn
(:101-112) writes the decoded image.  The reference reads PNGs with OpenCV
(IMREAD_UNCHANGED + BGR2RGB) and writes them with skimage.io.imsave; here
PIL does both (assumption A9: lossless 8-bit RGB PNG decode is the same
array either way; the PNG bytes written by decode_write_fn may differ from
skimage's encoder, the pixels do not).
"""
from __future__ import annotations

import logging
import os

import numpy as np


def _read_png_native(fn: str):
    """The library's PNG reader (vcf_amd/csrc/vcf_png.cpp): 8-bit, non-interlaced
    PNGs; None when the file is outside what it covers (PIL then reads it)."""
    import ctypes
    from .. import _lib
    with open(fn, "rb") as f:
        data = f.read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        return None, len(data)
    h, w, ok = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    buf = ctypes.c_char_p(data)
    _lib.call("vcf_png_info", buf, len(data), ctypes.byref(h), ctypes.byref(w), ctypes.byref(ok))
    if not ok.value:
        return None, len(data)
    img = np.empty((h.value, w.value, 3), np.uint8)
    _lib.call("vcf_png_decode_rgb", buf, len(data), img.ctypes.data_as(ctypes.c_void_p), img.nbytes)
    return img, len(data)


def read_image(fn: str) -> tuple[np.ndarray, int]:
    """(H x W x 3 uint8 RGB array, bytes on disk)."""
    if fn.lower().endswith(".png"):
        img, size = _read_png_native(fn)
        if img is not None:
            return img, size
    from PIL import Image
    size = os.path.getsize(fn)
    with Image.open(fn) as im:
        if im.mode in ("RGB", "RGBA", "P", "PA", "CMYK", "YCbCr"):
            img = np.asarray(im.convert("RGB"))
        elif im.mode in ("I;16", "I;16B", "I"):
            img = np.asarray(im)     # 16-bit: kept as is (the HIP path rejects it)
        else:
            img = np.asarray(im)
    return np.ascontiguousarray(img), size


PNG_LEVEL = 6        # zlib level of the PNGs written (PIL's / imageio's default)
PNG_THREADS = 16     # deflate pieces of one PNG in parallel (the box's CPU share)


def write_image(fn: str, img: np.ndarray) -> int:
    """Write img; H x W x 3 uint8 to .png goes through the library's parallel
    PNG writer (vcf_png_encode_rgb: pixel-exact), anything else through PIL."""
    a = np.ascontiguousarray(img)
    if fn.lower().endswith(".png") and a.ndim == 3 and a.shape[2] == 3 and a.dtype == np.uint8 and a.size:
        import ctypes
        from .. import _lib
        H, W = a.shape[:2]
        cap = int(_lib.lib().vcf_png_encode_bound(H, W))
        buf = np.empty(cap, np.uint8)
        n = ctypes.c_int64()
        import threading
        # frame-level worker threads already run in parallel: fewer deflate threads each
        th = PNG_THREADS if threading.current_thread() is threading.main_thread() else 2
        _lib.call("vcf_png_encode_rgb", a.ctypes.data_as(ctypes.c_void_p), H, W, PNG_LEVEL, th,
                  buf.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n))
        with open(fn, "wb") as f:
            f.write(memoryview(buf)[:n.value])
        return n.value
    from PIL import Image
    Image.fromarray(a).save(fn)
    return os.path.getsize(fn)


class CoDec:
    """entropy_image_coding.CoDec (:32-121), with the entropy stage injected."""

    file_extension = ""

    def __init__(self, args):
        logging.debug(f"trace args={args}")
        self.args = args
        self.encoding = getattr(args, "subparser_name", "encode") == "encode"
        self.total_input_size = 0
        self.total_output_size = 0

    def bye(self):
        logging.info(f"Input bytes = {self.total_input_size}")
        logging.info(f"Output bytes = {self.total_output_size}")

    def encode_read_fn(self, fn):
        img, input_size = read_image(fn)
        self.total_input_size += input_size
        logging.debug(f"Read {input_size} bytes from {fn} with shape {img.shape} and type={img.dtype}")
        self.img_shape = img.shape
        return img

    def encode_read(self, fn="/tmp/original.png"):
        return self.encode_read_fn(fn)

    def encode_write_fn(self, codestream, fn):
        codestream.seek(0)
        with open(fn + self.file_extension, "wb") as f:
            f.write(codestream.read())
        output_size = os.path.getsize(fn + self.file_extension)
        self.total_output_size += output_size
        logging.info(f"Written {output_size} bytes in {fn + self.file_extension}")
        return output_size

    def encode_write(self, codestream, fn="/tmp/encoded"):
        return self.encode_write_fn(codestream, fn)

    def decode_read_fn(self, fn):
        input_size = os.path.getsize(fn + self.file_extension)
        self.total_input_size += input_size
        with open(fn + self.file_extension, "rb") as f:
            return f.read()

    def decode_read(self, fn="/tmp/encoded"):
        return self.decode_read_fn(fn)

    def decode_write_fn(self, img, fn):
        output_size = write_image(fn, img)
        self.img_shape = img.shape
        self.total_output_size += output_size
        logging.debug(f"Written {output_size} bytes in {fn} with shape {img.shape} and type {img.dtype}")
        return output_size

    def decode_write(self, img, fn="/tmp/decoded.png"):
        return self.decode_write_fn(img, fn)
