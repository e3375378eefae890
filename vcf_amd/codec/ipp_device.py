"""IPP encode with the whole sequence resident in HBM: config C5's data path.

The reference's GOP loop (src/IPP_DCT.py:397-575, IPP.temporal_filter, no
RDO) codes, per GOP, an I-frame through encode_decode_proxy and then every
P-frame as motion search against the previous reconstruction
(_process_block_row :207-246), compensation (:378-395), the residual
cur - comp + 128 clipped (:547-551), the 2D-DCT codec round trip of the
residual (encode_fn -> .tif, decode_fn, :595-626) and the reconstruction
comp + rec - 128 clipped (:559-561).  GOPs are independent, frames inside a
GOP are serial.  Here a rank's GOPs (GOP g on rank floor(g*P/G),
shard.frame_range over GOPs) advance in lock step: at step p every GOP's
frame p is processed, the per-frame tools on each GOP's frame and the DCT +
deadzone encode and the DCT decode as one batched launch each over the step's
frames; every frame's indices stay in HBM, and after the loop all their TIFF
strips are deflated in one call (vcf_zlib_strips, byte-exact with zlib).
Nothing but the strip sizes and the motion fields leaves the GPU until the
end: then every frame's TIFF file (the host writer's prefix + the deflated
strips) is packed on the device and gathered to rank 0 over RCCL
(iii_device.Exchange), like config C4.

The files equal what vcf_amd.codec.ipp.CoDec writes for the same frames
(its encode_fn TIFFs), frame for frame; bench.py's c5 block checks frames
against the reference-loop restatement (tests/test_ipp_gpu.py::_ipp_loop).
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from .. import _lib
from .. import dct as D
from .. import zlib_gpu as Z
from ..device import DeviceBuffer, Stream, copy_dtod
from .iii_device import Exchange
from .shard import frame_range
from .tiff import container_prefixes, strip_layout


class _At:
    """A DeviceBuffer-like view: nbytes from byte `off` of another buffer."""

    def __init__(self, buf: DeviceBuffer, off: int, nbytes: int):
        self.ptr = buf.address(off)
        self.nbytes = int(nbytes)


class DeviceIPP:
    """One rank's part of a GOP-sharded, HBM-resident IPP encode (2D-DCT,
    deadzone Q, the reference's default -c TIFF), full search or --fast."""

    def __init__(self, comm, rank: int, world: int, n_frames: int, H: int, W: int, Q: int = 32, gop: int = 10,
                 bs: int = 16, sr: int = 8, fast: bool = False):
        self.comm, self.rank, self.world = comm, int(rank), int(world)
        self.N, self.H, self.W, self.Q = int(n_frames), int(H), int(W), int(Q)
        self.gop, self.bs, self.sr, self.fast = int(gop), int(bs), int(sr), bool(fast)
        self.n_gops = (self.N + self.gop - 1) // self.gop
        self.g_lo, self.g_hi = frame_range(self.n_gops, self.rank, self.world)

        def ranges(r):   # the frames of rank r's GOPs: one contiguous range
            glo, ghi = frame_range(self.n_gops, r, self.world)
            return min(glo * self.gop, self.N), min(ghi * self.gop, self.N)
        self.lo, self.hi = ranges(self.rank)
        self.n_local = self.hi - self.lo
        self.Hp, self.Wp = D.padded_shape(self.H, self.W)
        self.shape = (self.Hp, self.Wp, 3)
        self.fb, self.kb = self.H * self.W * 3, self.Hp * self.Wp * 3
        self.strip_bytes = strip_layout(self.shape, 1)[2]
        if not Z.covers(self.shape, 1):
            raise NotImplementedError(f"{self.Wp}-pixel rows: TIFF strips beyond the GPU deflate's")
        self.spf = Z.strip_count(self.kb, self.strip_bytes)
        self.slot = Z.bound(self.strip_bytes)
        self.hb, self.wb = self.H // self.bs, self.W // self.bs
        self.stream = Stream()
        ng = max(1, self.g_hi - self.g_lo)
        # per GOP: its reference and compensated frames; per step: the batch of residuals,
        # their indices and reconstructions (GOP order); every frame's strips and sizes
        self.ref = DeviceBuffer(ng * self.fb)
        self.comp = DeviceBuffer(ng * self.fb)
        self.res = DeviceBuffer(ng * self.fb)
        self.rec = DeviceBuffer(ng * self.fb)
        self.k = DeviceBuffer(max(1, self.n_local) * self.kb)   # every frame's indices, in deflate order
        # every local frame's motion field at its frame slot (the I-frames' slots unused): the
        # fields stay in HBM through the GOP loop and come back in one copy after it
        self.mvb = self.hb * self.wb * 8
        self.mv = DeviceBuffer(max(1, max(1, self.n_local) * self.mvb))
        self.gray = DeviceBuffer(2 * self.H * self.W)
        self.out = DeviceBuffer(max(1, self.n_local * self.spf * self.slot))
        self.sizes = DeviceBuffer(max(4, self.n_local * self.spf * 4))
        self.ws = Z.workspace_buffer(max(1, self.n_local) * self.spf)
        self.exchange = Exchange(comm, self.rank, self.world, self.N, ranges, self.stream)

    def _frames_of_step(self, p: int):
        """Local GOP indices g (0-based in this rank) that have a frame p."""
        return [g for g in range(self.g_hi - self.g_lo) if (self.g_lo + g) * self.gop + p < self.N]

    def run(self, frames: DeviceBuffer, stages: dict | None = None):
        """Encode this rank's frames (frames: n_local frames, H x W x 3 u8,
        back to back, global frames [lo, hi)) and gather every frame's TIFF on
        rank 0.  -> (sizes of all N files, rank 0's list of N memoryviews /
        None, this rank's motion fields: (P-frames, H/bs, W/bs, 2) float32 in
        frame order)."""
        call, sh = _lib.call, self.stream.handle
        fb, kb = self.fb, self.kb

        def mark(name, t0):
            if stages is None:
                return t0
            self.stream.synchronize()
            t1 = time.perf_counter()
            stages[name] = stages.get(name, 0.0) + (t1 - t0)
            return t1

        t = time.perf_counter()
        order = []   # local frame index (frame - lo) of each deflated frame, in deflate order
        p_frames = []   # local indices of the P-frames, whose motion fields come back
        for p in range(self.gop):
            gs = self._frames_of_step(p)
            if not gs:
                break
            for j, g in enumerate(gs):
                f = (self.g_lo + g) * self.gop + p - self.lo           # local frame index
                cur = _At(frames, f * fb, fb)
                if p == 0:   # the I-frame: coded as it is
                    copy_dtod(self.res, j * fb, frames, f * fb, fb, self.stream)
                    continue
                ref, comp = _At(self.ref, g * fb, fb), _At(self.comp, g * fb, fb)
                mv = _At(self.mv, f * self.mvb, self.mvb)
                call("vcf_ipp_block_match", ref.ptr, cur.ptr, self.H, self.W, self.bs, self.sr, int(self.fast),
                     mv.ptr, self.gray.ptr, sh)
                call("vcf_ipp_motion_compensate", ref.ptr, mv.ptr, self.H, self.W, self.bs, comp.ptr, sh)
                call("vcf_ipp_residual", cur.ptr, comp.ptr, fb, self.res.address(j * fb), sh)
                p_frames.append(f)
            n = len(gs)
            # the step's indices stay in HBM at their deflate positions [len(order), len(order) + n)
            kstep = _At(self.k, len(order) * kb, n * kb)
            D.encode_device(self.res, n, self.H, self.W, self.Q, 0, out=kstep, stream=self.stream)
            D.decode_device(kstep, n, self.H, self.W, self.Q, 0, out=self.rec, stream=self.stream)
            for j, g in enumerate(gs):
                rec = self.rec.address(j * fb)
                if p == 0:
                    copy_dtod(self.ref, g * fb, self.rec, j * fb, fb, self.stream)
                else:
                    call("vcf_ipp_reconstruct", self.comp.address(g * fb), rec, fb, self.ref.address(g * fb), sh)
                order.append((self.g_lo + g) * self.gop + p - self.lo)
        # every frame's TIFF strips in one call (one set of rounds instead of one partial
        # round per step: 10 calls of ~3 000 strips left the GPU half idle in each tail)
        if self.n_local:
            call("vcf_zlib_strips", self.k.ptr, self.n_local, kb, self.strip_bytes, Z.LEVEL, self.out.ptr, self.slot,
                 self.sizes.ptr, self.ws.ptr, sh)
        t = mark("gop_loop", t)
        # every frame's TIFF prefix from the strip sizes, the strips in frame order; the motion
        # fields of the whole loop in the same synchronisation
        sz = np.empty(max(1, self.n_local * self.spf), np.int32)
        if self.n_local:
            self.sizes.download(sz[:self.n_local * self.spf], self.stream)
        mv_all = np.empty((max(1, self.n_local), self.hb, self.wb, 2), np.float32)
        if self.n_local and self.mvb:
            call("vcf_memcpy_dtoh", mv_all.ctypes.data_as(ctypes.c_void_p), self.mv.ptr, self.n_local * self.mvb, sh)
        self.stream.synchronize()
        if (sz[:self.n_local * self.spf] < 0).any():
            raise RuntimeError("vcf_zlib_strips: a strip overflowed its slot")
        t = mark("sizes_d2h", t)
        pos = np.empty(self.n_local, np.int64)          # deflate position of local frame f
        pos[np.asarray(order, np.int64)] = np.arange(self.n_local)
        szf = sz[:self.n_local * self.spf].astype(np.int64).reshape(self.n_local, self.spf)[pos]
        hdr = container_prefixes(self.shape, np.uint8, szf) if self.n_local else np.zeros((0, 0), np.uint8)
        hlen = np.full(self.n_local, hdr.shape[1], np.int64)
        pay_src = (pos[:, None] * self.spf + np.arange(self.spf)[None, :]) * self.slot
        sizes, out = self.exchange.run(hdr.reshape(-1), hlen, self.out, pay_src, szf, mark, t)
        mvs = [mv_all[f] for f in sorted(p_frames)]
        return sizes, out, mvs
