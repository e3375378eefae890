"""GPU deflate of TIFF strips: the reference's default entropy stage
(TIFF.py:23-31, tifffile.imwrite(..., compression='zlib')) with the strips
deflated on the GPU, byte for byte what zlib.compress(strip, 6) returns
(libvcf_amd.so: vcf_zlib_strips; algorithm in csrc/vcf_deflate.h).

Frames already in HBM (the DCT/DWT kernels' index frames) are deflated where
they are; only the compressed strips come back: the per-strip streams are
packed on the device (vcf_copy_pieces) and copied to the host in one piece.
The TIFF file around them is vcf_amd.codec.tiff.container, the same writer
the host path uses, so the files are identical.
"""
from __future__ import annotations

import threading

import numpy as np

from . import _lib as L
from .device import DeviceBuffer, Stream, copy_pieces

LEVEL = 6   # tifffile 2021.7.2's zlib level (vcf_amd/codec/tiff.py ZLIB_LEVEL)


def strip_count(frame_bytes: int, strip_bytes: int) -> int:
    return int(L.lib().vcf_zlib_strip_count(int(frame_bytes), int(strip_bytes)))


def bound(strip_bytes: int) -> int:
    return int(L.lib().vcf_zlib_bound(int(strip_bytes)))


def workspace(n_strips: int) -> int:
    """Workspace bytes of one vcf_zlib_strips call over n_strips strips."""
    return int(L.lib().vcf_zlib_workspace(int(n_strips)))


def workspace_buffer(n_strips: int) -> DeviceBuffer:
    """A device workspace for a vcf_zlib_strips call over n_strips strips.
    When the library's default budget (a quarter of the memory free at first
    use, up to 40 GB) cannot be allocated -- the caller holds large buffers,
    or ranks share the device -- the budget is halved until it can: the
    strips then run in more rounds over a smaller workspace (same bytes, more
    time).  The new budget stays in effect for the device."""
    need, one = workspace(n_strips), workspace(1)
    while True:
        try:
            return DeviceBuffer(max(16, need))
        except L.VCFError:
            if need <= one:
                raise
            L.call("vcf_zlib_set_workspace_budget", max(one, need // 2))
            need = workspace(n_strips)


def max_strip() -> int:
    """The largest strip the GPU deflate takes (vcf_zlib_max_strip: 65536 bytes)."""
    return int(L.lib().vcf_zlib_max_strip())


def covers(shape, itemsize: int = 1) -> bool:
    """True when tifffile's strips of an H x W [x C] array fit the GPU deflate
    (rows of at most 64 KB; wider frames keep the host TIFF writer)."""
    from .codec.tiff import strip_layout
    shape = tuple(int(s) for s in shape)
    return strip_layout(shape if len(shape) == 3 else shape + (1,), itemsize)[2] <= max_strip()


class StripDeflater:
    """Deflates every strip of a batch of device-resident frames.  Scratch
    buffers grow on demand and are reused; calls are serialised (one set of
    scratch, one stream)."""

    def __init__(self):
        self._bufs = {}
        self._stream = None
        self._lock = threading.Lock()

    def _buf(self, name: str, nbytes: int) -> DeviceBuffer:
        b = self._bufs.get(name)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
            b = self._bufs[name] = DeviceBuffer(max(int(nbytes), 16))
        return b

    def _workspace(self) -> DeviceBuffer:
        ws = self._bufs.get("ws")
        if ws is not None and ws.nbytes >= workspace(self.total):
            return ws
        if ws is not None:
            ws.free()
            del self._bufs["ws"]
        ws = self._bufs["ws"] = workspace_buffer(self.total)
        return ws

    def launch(self, src: DeviceBuffer, n_frames: int, frame_bytes: int, strip_bytes: int, level: int = LEVEL,
               offset: int = 0, stream: Stream | None = None) -> None:
        """Queue the deflate of every strip on `stream` (default: the
        deflater's own); strip s's stream then sits at byte s * slot of
        `out`.  sizes() waits for it.  The caller holds the deflater (one
        batch at a time)."""
        if stream is None:
            if self._stream is None:
                self._stream = Stream()
            stream = self._stream
        self.stream = stream
        self.spf = strip_count(frame_bytes, strip_bytes)
        self.n_frames = int(n_frames)
        self.total = self.spf * self.n_frames
        self.slot = bound(strip_bytes)
        if self.total == 0:
            return
        self.out = self._buf("out", self.total * self.slot)
        self._sizes = self._buf("sizes", self.total * 4)
        ws = self._workspace()
        L.call("vcf_zlib_strips", src.address(offset), int(n_frames), int(frame_bytes), int(strip_bytes),
               int(level), self.out.ptr, self.slot, self._sizes.ptr, ws.ptr, stream.handle)

    def sizes(self) -> np.ndarray:
        """Compressed size of every strip of the last launch (int32, frame-major)."""
        sz = np.empty(self.total, np.int32)
        if self.total:
            self._sizes.download(sz, self.stream)
        self.stream.synchronize()
        if (sz < 0).any():
            raise RuntimeError("vcf_zlib_strips: a strip overflowed its slot")
        return sz

    def deflate_device(self, src: DeviceBuffer, n_frames: int, frame_bytes: int, strip_bytes: int,
                       level: int = LEVEL, offset: int = 0, stream: Stream | None = None):
        """-> list over frames of lists of strip streams (bytes).  `src` holds
        n_frames frames of frame_bytes bytes from byte `offset`; work on
        `stream` (default: the deflater's own) is complete before the call
        returns."""
        with self._lock:
            self.launch(src, n_frames, frame_bytes, strip_bytes, level, offset, stream)
            total, spf, slot, stream = self.total, self.spf, self.slot, self.stream
            if total == 0:
                return [[] for _ in range(int(n_frames))]
            sz = self.sizes()
            # pack the streams on the device, one download
            offs = np.zeros(total + 1, np.int64)
            np.cumsum(sz, out=offs[1:])
            table = np.empty((total, 3), np.int64)
            table[:, 0] = np.arange(total, dtype=np.int64) * slot
            table[:, 1] = offs[:-1]
            table[:, 2] = sz
            tb = self._buf("table", table.nbytes)
            tb.upload(table, stream)
            packed = self._buf("packed", int(offs[-1]))
            copy_pieces(self.out, tb, total, packed, stream)
            host = np.empty(int(offs[-1]), np.uint8)
            if host.size:
                packed.download(host, stream)
            stream.synchronize()
            blob = host.tobytes()
            return [[blob[offs[f * spf + k]:offs[f * spf + k + 1]] for k in range(spf)] for f in range(int(n_frames))]

    def close(self):
        for b in self._bufs.values():
            b.free()
        self._bufs.clear()


_default = None


def deflater() -> StripDeflater:
    global _default
    if _default is None:
        _default = StripDeflater()
    return _default


def tiff_frames_device(src: DeviceBuffer, n_frames: int, shape, dtype=np.uint8, offset: int = 0,
                       stream: Stream | None = None) -> list:
    """TIFF files (bytes) of n_frames device-resident H x W [x C] u8/u16
    arrays, identical to vcf_amd.codec.tiff.imwrite_bytes of each (TIFF.py:29)."""
    from .codec.tiff import container, strip_layout
    dt = np.dtype(dtype)
    if dt not in (np.uint8, np.uint16):
        raise ValueError(f"current type = {dt}")   # TIFF.py:27
    shape = tuple(int(s) for s in shape)
    frame_bytes = int(np.prod(shape)) * dt.itemsize
    _, _, strip_bytes = strip_layout(shape if len(shape) == 3 else shape + (1,), dt.itemsize)
    strips = deflater().deflate_device(src, n_frames, frame_bytes, strip_bytes, LEVEL, offset, stream)
    return [container(shape, dt, s) for s in strips]


class StripInflater:
    """zlib.decompress of a batch of strips on the GPU (vcf_inflate_strips), the
    decode side of TIFF.py:33-39: the compressed strips go up in one copy, the
    inflated bytes land in a device buffer (e.g. the index frames the DCT
    decode reads).  Buffers grow on demand and are reused."""

    def __init__(self):
        self._bufs = {}
        self._lock = threading.Lock()

    def _buf(self, name: str, nbytes: int) -> DeviceBuffer:
        b = self._bufs.get(name)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
            b = self._bufs[name] = DeviceBuffer(max(int(nbytes), 16))
        return b

    def inflate_into(self, comp: np.ndarray, comp_off: np.ndarray, comp_len: np.ndarray, out: DeviceBuffer,
                     out_off: np.ndarray, out_len: np.ndarray, stream: Stream, violations: np.ndarray = None) -> None:
        """Strip s: comp[comp_off[s]:][:comp_len[s]] (host bytes) -> out at
        out_off[s], exactly out_len[s] bytes.  Raises ValueError naming the
        first strip zlib would reject (corrupt stream, wrong length, adler32),
        and before anything runs on the device for a strip table that does not
        fit its buffers (a negative length, a strip past the end of `comp` or
        of `out`).  With `violations` (a uint32 array of one entry per strip)
        the strips run through the A/B library's window-check diagnostic
        (vcf_inflate_strips_wincheck), which fills it; test use only."""
        n = int(len(comp_len))
        comp = np.ascontiguousarray(comp, np.uint8)
        comp_off, out_off = np.asarray(comp_off, np.int64), np.asarray(out_off, np.int64)
        comp_len, out_len = np.asarray(comp_len, np.int64), np.asarray(out_len, np.int64)
        if not (len(comp_off) == len(out_off) == len(out_len) == n):
            raise ValueError("inflate: strip table arrays of different lengths")
        if n == 0:
            return
        if (comp_len < 0).any() or (out_len < 0).any() or (comp_off < 0).any() or (out_off < 0).any():
            raise ValueError("inflate: negative strip offset or length")
        if (comp_off + comp_len > comp.nbytes).any():
            raise ValueError(f"inflate: strip {int(np.argmax(comp_off + comp_len > comp.nbytes))} reads past the "
                             f"{comp.nbytes} compressed bytes")
        if (out_off + out_len > out.nbytes).any() or (out_len > 0x7FFFFFFF).any() or (comp_len > 0x7FFFFFFF).any():
            raise ValueError(f"inflate: a strip writes past the {out.nbytes}-byte output buffer")
        tab = np.concatenate([comp_off, out_off])
        lens = np.concatenate([comp_len, out_len]).astype(np.int32)
        with self._lock:
            dc, dt, dl, ds = (self._buf("comp", comp.nbytes), self._buf("tab", tab.nbytes),
                              self._buf("lens", lens.nbytes), self._buf("status", 4 * n))
            dc.upload(comp, stream)
            dt.upload(tab, stream)
            dl.upload(lens, stream)
            if violations is None:
                L.call("vcf_inflate_strips", dc.ptr, dt.ptr, dl.ptr, n, out.ptr, dt.address(8 * n),
                       dl.address(4 * n), ds.ptr, stream.handle)
            else:
                dv = self._buf("viol", 4 * n)
                L.call_ab("vcf_inflate_strips_wincheck", dc.ptr, dt.ptr, dl.ptr, n, out.ptr, dt.address(8 * n),
                          dl.address(4 * n), ds.ptr, dv.ptr, stream.handle)
                dv.download(violations[:n], stream)
            st = np.empty(n, np.int32)
            ds.download(st, stream)
            stream.synchronize()
        bad = np.nonzero(st)[0]
        if bad.size:
            raise ValueError(f"inflate: strip {int(bad[0])} is not a zlib stream of its length (status {int(st[bad[0]])})")

    def close(self):
        for b in self._bufs.values():
            b.free()
        self._bufs.clear()


_inflater = None


def inflater() -> StripInflater:
    global _inflater
    if _inflater is None:
        _inflater = StripInflater()
    return _inflater
