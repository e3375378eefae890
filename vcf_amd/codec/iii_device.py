"""III encode with every frame resident in HBM: config C4's data path.

The reference's III loop (src/III.py:77-115) runs encode_fn frame after frame
in one process: read PNG, 2D-DCT + deadzone (2D-DCT.py:276-361), entropy
code, write /tmp/encoded_%04d.  Here a sequence of N frames is sharded over
P ranks (frame i on rank floor(i*P/N), shard.frame_range) and each rank's
chunk never leaves the GPU until its code-streams are final:

  1. one launch of the fused DCT + deadzone kernel over the rank's chunk
     (vcf_dct_dz_encode), indices stay in HBM;
  2. the GPU entropy stage, all frames in one launch per stage, only the
     small size tables coming to the host: either every frame's indices
     coded as a prior-seeded tiled CBAAC stream (`-c TCBAACP`,
     vcf_amd/tcbaac.py), or -- the reference's default `-c TIFF` -- every
     TIFF strip of every frame deflated exactly as zlib would
     (vcf_amd/zlib_gpu.py);
  3. every frame's file (header + payload: exactly the bytes
     `TiledCBAACCodec.compress_device`, resp. the TIFF writer, returns for
     it) is assembled in a device send buffer;
  4. the exchange: per-frame container sizes all-gathered
     (ncclAllGather), the containers gathered to rank 0 device to device
     (vcf_comm_gatherv: one ncclSend per peer, P-1 receives on rank 0, each
     over its own xGMI link), then one copy to rank 0's host.

No PyTorch; RCCL through libvcf_amd.so (vcf_amd/rccl.py), bounded by its
timeouts.  bench.py reports this as its C4 block next to the kernel
headline.
"""
from __future__ import annotations

import time

import numpy as np

from .. import dct as D
from .. import tcbaac as T
from .. import zlib_gpu as Z
from ..device import DeviceBuffer, HostBuffer, Stream, copy_dtod, copy_pieces
from .shard import frame_range
from .tiff import container_prefixes, strip_layout


class DeviceIII:
    """One rank's part of a frame-sharded, HBM-resident III encode."""

    def __init__(self, comm, rank: int, world: int, n_frames: int, H: int, W: int, Q: int = 32,
                 seg_len: int = T.CLASS_SEG, streams: int = 4, nclass: int = T.PRIOR_CLASSES,
                 entropy: str = "TCBAACP"):
        self.comm, self.rank, self.world = comm, int(rank), int(world)
        self.N, self.H, self.W, self.Q = int(n_frames), int(H), int(W), int(Q)
        self.lo, self.hi = frame_range(self.N, self.rank, self.world)
        self.n_local = self.hi - self.lo
        self.Hp, self.Wp = D.padded_shape(self.H, self.W)
        self.shape = (self.Hp, self.Wp, 3)
        self.n_sym = self.Hp * self.Wp * 3
        self.stream = Stream()
        self.k = DeviceBuffer(max(self.n_local * self.n_sym, 1))
        if entropy not in ("TCBAACP", "TIFF"):
            raise ValueError(f"entropy codec {entropy!r}: TCBAACP or TIFF")
        self.entropy = entropy
        if entropy == "TIFF":
            self.batch = None
            self.zd = Z.StripDeflater()
            self.strip_bytes = strip_layout(self.shape, 1)[2]
            if not Z.covers(self.shape, 1):
                raise NotImplementedError(f"{self.Wp}-pixel rows: TIFF strips of {self.strip_bytes} bytes are beyond "
                                          f"the GPU deflate's {Z.max_strip()}; use the file path (dct2d.encode_fns)")
        else:
            self.batch = T.FrameBatch(self.n_local, self.n_sym, 0, seg_len, prior=True, nclass=nclass)
        self.exchange = Exchange(comm, self.rank, self.world, self.N, lambda r: frame_range(self.N, r, self.world),
                                 self.stream)

    def run(self, rgb: DeviceBuffer, stages: dict | None = None):
        """Encode this rank's frames (rgb: n_local frames, H x W x 3 u8, back
        to back) and gather every frame's container on rank 0.
        -> (per-frame container sizes of all N frames, list of N containers on
        rank 0 -- memoryviews into the page-locked receive buffer, valid until
        the next run -- / None elsewhere).  With `stages`, each stage is
        synchronised and its seconds are added under its name (diagnostic:
        the syncs cost a little)."""
        def mark(name, t0):
            if stages is None:
                return t0
            self.stream.synchronize()
            t1 = time.perf_counter()
            stages[name] = stages.get(name, 0.0) + (t1 - t0)
            return t1

        t = time.perf_counter()
        if self.n_local:
            D.encode_device(rgb, self.n_local, self.H, self.W, self.Q, 0, out=self.k, stream=self.stream)
        t = mark("dct_dz", t)
        if self.entropy == "TIFF":
            # the TIFF files: header (built on the host from the strip sizes) + the strips as deflated
            if self.n_local:
                self.zd.launch(self.k, self.n_local, self.n_sym, self.strip_bytes, Z.LEVEL, 0, self.stream)
                sz = self.zd.sizes().astype(np.int64).reshape(self.n_local, -1)
            else:
                sz = np.zeros((0, 1), np.int64)
            t = mark("entropy", t)
            # every frame's TIFF prefix at once (only the strip offsets / byte counts differ)
            hdr = container_prefixes(self.shape, np.uint8, sz) if self.n_local else np.zeros((0, 0), np.uint8)
            hlen = np.full(self.n_local, hdr.shape[1], np.int64)
            hb = hdr.reshape(-1)
            pay_buf = self.zd.out if self.n_local else None
            spf = sz.shape[1]
            pay_src = (np.arange(self.n_local * spf, dtype=np.int64) * self.zd.slot if self.n_local else
                       np.zeros(0, np.int64)).reshape(self.n_local, spf)
            pay_len = sz
        else:
            if self.n_local:
                self.batch.launch(self.k, after=self.stream)
            seg, totals, priors = self.batch.sizes()          # waits for the coder
            t = mark("entropy", t)
            headers = self.batch.headers(self.shape)
            hlen = np.array([len(h) for h in headers], np.int64)
            hb = np.frombuffer(b"".join(headers), np.uint8)
            pay_buf = self.batch.out
            pay_src = np.zeros((self.n_local, 1), np.int64)
            pay_len = np.zeros((self.n_local, 1), np.int64)
            for f in range(self.n_local):
                pbuf, poff, pn = self.batch.payload(f)
                pay_src[f, 0], pay_len[f, 0] = poff, pn
        return self.exchange.run(hb, hlen, pay_buf, pay_src, pay_len, mark, t)


class Exchange:
    """The containers of one rank's frames packed into a device send buffer
    and gathered to rank 0: per-frame sizes all-gathered
    (ncclAllGather), the containers gathered device to device
    (vcf_comm_gatherv: one ncclSend per peer, each over its own xGMI link),
    then one copy to rank 0's page-locked host buffer.  Rank r holds the
    global frames ranges(r) = [lo, hi) (contiguous, rank order)."""

    def __init__(self, comm, rank: int, world: int, N: int, ranges, stream: Stream):
        self.comm, self.rank, self.world, self.N = comm, int(rank), int(world), int(N)
        self.ranges = ranges
        self.lo, self.hi = ranges(self.rank)
        self.n_local = self.hi - self.lo
        self.stream = stream
        self.send = self.recv = self.hstage = self.table = self.host = None

    def _buf(self, name: str, nbytes: int) -> DeviceBuffer:
        b = getattr(self, name)
        if b is None or b.nbytes < nbytes:
            b = DeviceBuffer(max(nbytes, 1))
            setattr(self, name, b)
        return b

    def run(self, hb: np.ndarray, hlen: np.ndarray, pay_buf, pay_src: np.ndarray, pay_len: np.ndarray, mark, t):
        """hb: every local frame's header bytes back to back (hlen[f] each);
        frame f's payload is pay_len[f, j] bytes at pay_src[f, j] of pay_buf,
        j in order.  -> (sizes of all N containers, rank 0's list of N
        memoryviews into the page-locked receive buffer / None)."""
        local_sizes = hlen + pay_len.sum(axis=1)
        nbytes = int(local_sizes.sum())
        send = self._buf("send", nbytes)
        if self.n_local:
            # headers (staged from the host) and payloads (in the coder's output)
            # land back to back in the send buffer: two gather-copy launches, their
            # piece tables computed in whole arrays
            hst = self._buf("hstage", hb.size)
            hst.upload(hb, self.stream)
            npay = pay_len.shape[1]
            frame_off = np.concatenate([[0], np.cumsum(local_sizes)[:-1]])
            hdr_tab = np.stack([np.concatenate([[0], np.cumsum(hlen)[:-1]]), frame_off, hlen], axis=1)
            pay_dst = (frame_off + hlen)[:, None] + np.concatenate(
                [np.zeros((self.n_local, 1), np.int64), np.cumsum(pay_len, axis=1)[:, :-1]], axis=1)
            pay_tab = np.stack([pay_src, pay_dst, pay_len], axis=2)
            tab = np.concatenate([hdr_tab.ravel(), pay_tab.ravel()]).astype(np.int64)
            tb = self._buf("table", tab.nbytes)
            tb.upload(tab, self.stream)
            copy_pieces(hst, tb, self.n_local, send, self.stream)
            copy_pieces(pay_buf, _View(tb, hdr_tab.nbytes), self.n_local * npay, send, self.stream)
        t = mark("pack", t)
        sizes = self._all_gather_sizes(local_sizes)
        t = mark("sizes_allgather", t)
        counts = np.array([sizes[slice(*self.ranges(r))].sum() for r in range(self.world)], np.int64)
        total = int(counts.sum())
        recv = self._buf("recv", total) if self.rank == 0 else None
        if self.comm is not None:
            self.comm.gatherv_device(send, nbytes, counts, recv, root=0, stream=self.stream)
            self.comm.wait(self.stream)
        elif nbytes:
            copy_dtod(recv, 0, send, 0, nbytes, self.stream)
        t = mark("gatherv", t)
        out = None
        if self.rank == 0:
            if self.host is None or self.host.nbytes < total:
                self.host = HostBuffer(total)   # page-locked: the gathered bytes come back at full PCIe speed
            blob = self.host.array[:total]
            if total:
                recv.download(blob, self.stream)
            self.stream.synchronize()
            # views into the page-locked buffer (valid until the next run), no per-frame copies
            mv = memoryview(blob)
            ends = np.cumsum(sizes)
            out = [mv[int(e - s):int(e)] for s, e in zip(sizes, ends)]
        else:
            self.stream.synchronize()
        mark("d2h_rank0", t)
        return sizes, out

    def _all_gather_sizes(self, local_sizes: np.ndarray) -> np.ndarray:
        full = np.zeros(self.N, np.int64)
        full[self.lo:self.hi] = local_sizes
        if self.comm is None or self.world == 1:
            return full
        rows = self.comm.all_gather_i64(full)
        out = np.zeros(self.N, np.int64)
        for r in range(self.world):
            rlo, rhi = self.ranges(r)
            out[rlo:rhi] = rows[r, rlo:rhi]
        return out


class _View:
    """A DeviceBuffer-like view `off` bytes into another (what vcf_copy_pieces takes)."""

    def __init__(self, buf: DeviceBuffer, off: int):
        self.ptr = buf.address(off)
