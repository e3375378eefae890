"""TIFF entropy codec: src/TIFF.py of the reference (TIFF.CoDec.compress /
decompress, :23-39), which calls tifffile.imwrite(..., compression='zlib')
and tifffile.imread.

The writer reproduces, byte for byte, what the reference's pinned tifffile
(2021.7.2, stdlib-zlib path, no imagecodecs) writes for a uint8/uint16
H x W x C array: classic little-endian TIFF, one IFD at offset 8 with 15
tags, out-of-line values in tag order (word aligned; the ImageDescription
slot keeps 16 spare bytes so tifffile can rewrite the shape), strip data
16-byte aligned, RowsPerStrip = 65536 // (W * C * itemsize) (at least 1),
each strip deflated on its own at zlib level 6 (tifffile's default level).
Strips are independent, so they are compressed on a thread pool -- zlib
releases the GIL (per-strip parallel deflate).

The reader accepts any baseline TIFF the reference could produce or read
(uncompressed or Adobe-deflate strips, chunky 8/16-bit samples, either byte
order), which covers the libdeflate-made files of the imagecodecs path too.
"""
from __future__ import annotations

import io
import json
import os
import struct
import threading
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ZLIB_LEVEL = 6          # tifffile 2021.7.2 zlib_encode default
_SOFTWARE = b"tifffile.py\x00"
_TYPE_SIZE = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 1, 7: 1, 8: 2, 9: 4, 10: 8, 11: 4, 12: 8, 16: 8}
_pool = None


def _executor():
    global _pool
    if _pool is None:
        _pool = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1))
    return _pool


def _deflate_strips(data: memoryview, strip_bytes: int, nstrips: int, level: int):
    chunks = [data[i * strip_bytes:(i + 1) * strip_bytes] for i in range(nstrips)]
    # strips in parallel only for a caller on the main thread: frame-level
    # worker threads (the III pipeline) already keep every core busy
    if nstrips >= 4 and len(data) >= (1 << 20) and threading.current_thread() is threading.main_thread():
        return list(_executor().map(lambda c: zlib.compress(c, level), chunks))
    return [zlib.compress(c, level) for c in chunks]


def strip_layout(shape, itemsize: int = 1):
    """(rows per strip, strips, bytes per full strip) tifffile 2021.7.2 uses
    for an H x W [x C] array: RowsPerStrip = 65536 // row bytes, at least 1."""
    H, W = shape[0], shape[1]
    C = shape[2] if len(shape) > 2 else 1
    row_bytes = W * C * itemsize
    rps = max(1, min(H, 65536 // max(1, row_bytes)))
    return rps, (H + rps - 1) // rps, rps * row_bytes


def imwrite_bytes(img: np.ndarray, level: int = ZLIB_LEVEL) -> bytes:
    """tifffile.imwrite(BytesIO, img, compression='zlib') for HxWxC u8/u16."""
    a = np.ascontiguousarray(img)
    if a.dtype not in (np.uint8, np.uint16):
        raise ValueError(f"current type = {a.dtype}")   # TIFF.py:27 asserts u8/u16
    if a.dtype.byteorder == ">":
        a = a.astype(a.dtype.newbyteorder("<"))
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim != 3:
        raise ValueError("TIFF writer expects an H x W [x C] array")
    rps, nstrips, strip_bytes = strip_layout(a.shape, a.dtype.itemsize)
    comp = _deflate_strips(memoryview(a.reshape(-1).view(np.uint8)), strip_bytes, nstrips, level)
    return container(img.shape, a.dtype, comp)


def container(shape, dtype, comp) -> bytes:
    """The TIFF file around already-deflated strips (tifffile's byte layout)."""
    return container_prefix(shape, dtype, [len(c) for c in comp]) + b"".join(comp)


def container_prefix(shape, dtype, counts) -> bytes:
    """Every byte of the TIFF file before its strip data (header, IFD, tag
    values, padding to the 16-byte aligned data offset), for strips of the
    given compressed sizes stored back to back after it."""
    H, W = shape[0], shape[1]
    C = shape[2] if len(shape) > 2 else 1
    isz = np.dtype(dtype).itemsize
    rps, nstrips, _ = strip_layout((H, W, C), isz)
    counts = [int(c) for c in counts]
    if len(counts) != nstrips:
        raise ValueError(f"{len(counts)} strips for a {H}x{W}x{C} image, expected {nstrips}")

    desc = json.dumps({"shape": list(shape)}).encode() + b"\x00"
    photometric = 2 if C == 3 else 1      # RGB for 3 samples, else minisblack
    tags = []   # (code, type, count, payload bytes or int)
    tags.append((256, 4, 1, W))
    tags.append((257, 4, 1, H))
    tags.append((258, 3, C, struct.pack("<%dH" % C, *([8 * isz] * C))))
    tags.append((259, 3, 1, 8))
    tags.append((262, 3, 1, photometric))
    tags.append((270, 2, len(desc), desc))
    tags.append((273, 4, nstrips, None))     # filled once the data offset is known
    tags.append((277, 3, 1, C))
    tags.append((278, 4, 1, rps))
    tags.append((279, 4, nstrips, struct.pack("<%dI" % nstrips, *counts) if nstrips > 1 else counts[0]))
    tags.append((282, 5, 1, struct.pack("<II", 1, 1)))
    tags.append((283, 5, 1, struct.pack("<II", 1, 1)))
    tags.append((284, 3, 1, 1))
    tags.append((296, 3, 1, 1))
    tags.append((305, 2, len(_SOFTWARE), _SOFTWARE))

    ifd_off = 8
    pos = ifd_off + 2 + 12 * len(tags) + 4
    # out-of-line values, in tag order, word aligned; the description keeps 16 spare bytes
    slots = {}
    for code, typ, count, payload in tags:
        size = _TYPE_SIZE[typ] * count
        if size <= 4:
            continue
        slots[code] = pos
        reserve = size + (16 if code == 270 else 0)
        pos += reserve + (reserve & 1)
    data_off = (pos + 15) & ~15
    offsets = [data_off]
    for c in counts[:-1]:
        offsets.append(offsets[-1] + c)

    out = bytearray(b"II*\x00" + struct.pack("<I", ifd_off))
    out += struct.pack("<H", len(tags))
    ool = bytearray(pos - (ifd_off + 2 + 12 * len(tags) + 4))
    base = ifd_off + 2 + 12 * len(tags) + 4
    for code, typ, count, payload in tags:
        if code == 273:
            payload = struct.pack("<%dI" % nstrips, *offsets) if nstrips > 1 else offsets[0]
        size = _TYPE_SIZE[typ] * count
        if size <= 4:
            if isinstance(payload, int):
                val = struct.pack("<H", payload) + b"\x00\x00" if typ == 3 else struct.pack("<I", payload)
            else:
                val = payload.ljust(4, b"\x00")
            out += struct.pack("<HHI", code, typ, count) + val
        else:
            off = slots[code]
            ool[off - base:off - base + size] = payload
            out += struct.pack("<HHII", code, typ, count, off)
    out += struct.pack("<I", 0)
    out += ool
    out += b"\x00" * (data_off - len(out))
    return bytes(out)


def container_prefixes(shape, dtype, counts) -> np.ndarray:
    """container_prefix for a batch of equal-shaped frames at once: counts is
    (n_frames, strips) compressed sizes -> (n_frames, prefix bytes) uint8, row
    f equal to container_prefix(shape, dtype, counts[f]).  Only the
    StripOffsets / StripByteCounts values differ between the frames, so the
    prefix is built once and those two arrays are filled in vectorised."""
    counts = np.asarray(counts, np.int64)
    n, ns = counts.shape
    tmpl = container_prefix(shape, dtype, [0] * ns)
    data_off = len(tmpl)
    nt = struct.unpack("<H", tmpl[8:10])[0]
    pos = {}
    for i in range(nt):
        e = 10 + 12 * i
        code, _, count = struct.unpack("<HHI", tmpl[e:e + 8])
        if code in (273, 279):
            pos[code] = e + 8 if 4 * count <= 4 else struct.unpack("<I", tmpl[e + 8:e + 12])[0]
    out = np.tile(np.frombuffer(tmpl, np.uint8), (n, 1))
    offs = np.full((n, ns), data_off, np.int64)
    offs[:, 1:] += np.cumsum(counts[:, :-1], axis=1)
    for code, v in ((273, offs), (279, counts)):
        out[:, pos[code]:pos[code] + 4 * ns] = v.astype("<u4").view(np.uint8).reshape(n, 4 * ns)
    return out


def _read_ifd(buf: bytes):
    bo = {b"II": "<", b"MM": ">"}.get(buf[:2])
    if bo is None or struct.unpack(bo + "H", buf[2:4])[0] != 42:
        raise ValueError("not a classic TIFF file")
    off = struct.unpack(bo + "I", buf[4:8])[0]
    n = struct.unpack(bo + "H", buf[off:off + 2])[0]
    fmt = {1: "B", 2: "s", 3: "H", 4: "I", 5: "II", 6: "b", 8: "h", 9: "i", 16: "Q"}
    tags = {}
    for i in range(n):
        e = off + 2 + 12 * i
        code, typ, count = struct.unpack(bo + "HHI", buf[e:e + 8])
        size = _TYPE_SIZE.get(typ, 1) * count
        raw = buf[e + 8:e + 8 + size] if size <= 4 else \
            buf[struct.unpack(bo + "I", buf[e + 8:e + 12])[0]:][:size]
        if typ == 2:
            tags[code] = raw.rstrip(b"\x00")
        elif typ in fmt:
            f = fmt[typ]
            vals = struct.unpack(bo + f * count, raw)
            tags[code] = vals
    return bo, tags


def tiff_strips(buf: bytes):
    """The strip table of a deflate-compressed, chunky, little-endian u8/u16
    TIFF (what tifffile writes for TIFF.py:29): (shape, dtype, strip offsets,
    strip byte counts, uncompressed bytes per full strip), or None for any
    other TIFF (imread_bytes reads those on the host) -- including one whose
    strip table does not describe the image: a strip count other than
    ceil(frame bytes / strip bytes), or a strip past the end of the file.
    The GPU inflate trusts the table it is given, so only a consistent one
    goes there; the host reader reports the others as zlib/tifffile would."""
    try:
        # the IFD of a tifffile-written file sits in the first 64 KiB; parse
        # the whole buffer when it does not (other writers put it at the end)
        try:
            bo, t = _read_ifd(bytes(buf[:65536]) if len(buf) > 65536 else bytes(buf))
        except (struct.error, ValueError, KeyError):
            if len(buf) <= 65536:
                raise
            bo, t = _read_ifd(bytes(buf))
    except (struct.error, ValueError, KeyError):
        return None
    if bo != "<" or t.get(259, (1,))[0] not in (8, 32946) or t.get(284, (1,))[0] != 1:
        return None
    if 273 not in t or 279 not in t or 256 not in t or 257 not in t:
        return None
    W, H = t[256][0], t[257][0]
    C = t.get(277, (1,))[0]
    bps = t.get(258, (8,))[0]
    if bps not in (8, 16) or W <= 0 or H <= 0 or C <= 0:
        return None
    isz = bps // 8
    rps = t.get(278, (H,))[0]
    shape = (H, W, C) if C > 1 else (H, W)
    strip_bytes = min(max(rps, 1), H) * W * C * isz
    offs, counts = list(t[273]), list(t[279])
    frame_bytes = H * W * C * isz
    if len(offs) != len(counts) or len(offs) != -(-frame_bytes // strip_bytes):
        return None
    if any(o < 0 or c < 0 or o + c > len(buf) for o, c in zip(offs, counts)):
        return None
    return shape, np.dtype("<u%d" % isz), offs, counts, strip_bytes


def imread_bytes(buf: bytes) -> np.ndarray:
    """tifffile.imread(BytesIO(buf)) for the files TIFF.py writes."""
    bo, t = _read_ifd(bytes(buf))
    W, H = t[256][0], t[257][0]
    C = t.get(277, (1,))[0]
    bps = t.get(258, (8,))[0]
    comp = t.get(259, (1,))[0]
    if t.get(284, (1,))[0] != 1:
        raise ValueError("planar TIFF not supported")
    dtype = np.dtype({8: "u1", 16: "u2"}[bps]).newbyteorder(bo)
    raw = bytearray()
    for o, c in zip(t[273], t[279]):
        s = buf[o:o + c]
        if comp in (8, 32946):
            s = zlib.decompress(s)
        elif comp != 1:
            raise ValueError(f"TIFF compression {comp} not supported")
        raw += s
    a = np.frombuffer(bytes(raw), dtype=dtype, count=H * W * C).astype(dtype.newbyteorder("="))
    return a.reshape((H, W, C) if C > 1 else (H, W))


class TIFFCodec:
    """The reference's TIFF entropy stage: compress(ndarray) -> BytesIO
    (seeked to 0, TIFF.py:23-31), decompress(bytes) -> ndarray (:33-39)."""
    # batches of frames whose indices sit in HBM (dct2d.CoDec.encode_fns) deflate
    # their strips on the GPU, byte-exact with zlib (vcf_amd/zlib_gpu.py)
    gpu_batches = True

    file_extension = ".tif"

    def compress(self, img: np.ndarray) -> io.BytesIO:
        assert img.dtype in (np.uint8, np.uint16), f"current type = {img.dtype}"
        b = io.BytesIO(imwrite_bytes(img))
        b.seek(0)
        return b

    def decompress(self, compressed_img) -> np.ndarray:
        if isinstance(compressed_img, io.BytesIO):
            compressed_img = compressed_img.getvalue()
        return imread_bytes(compressed_img)
