"""Tiled CBAAC: the CBAAC entropy stage (src/CBAAC.py) as a GPU-resident coder.

The reference codes a frame's indices as one serial arithmetic-coded stream
(CBAAC.py:114-131).  Here the flattened symbols split into consecutive
segments of `seg_len` symbols and every segment is coded exactly as the
reference codes a stream -- fresh AdaptiveModel/ContextManager, history of
`order` zeros, the A8 coder flushed at the segment's end -- one wave per
segment on the GPU (libvcf_amd.so: vcf_cbaac_tiled_*).  Segment i's bytes
equal vcf_cbaac_encode(symbols[i*seg_len:(i+1)*seg_len]).  The price is one
model warm-up per segment (the rate overhead, reported by
scripts/bench_tcbaac.py); the gain is that the frame's indices never leave
HBM -- only the compressed bytes come back.

Container (`.tadpt_arith`, a new format; the reference's `.adpt_arith` has
no segment index):
    uint32 ndims, uint32 shape[ndims]         (as CBAAC.py:84-89)
    b"VCFT", uint32 version = 1, uint32 order, uint32 seg_len,
    uint32 n_segments, uint32 segment_bytes[n_segments]
    the segments' bit streams, back to back (each MSB-first, zero padded)
Version 2 (`prior=True`, orders 0 and 1; not in the reference) adds, after
n_segments, 256 uint16 prior frequencies f[s] = 1 + floor(hist[s] * 8192 / n)
of the frame's symbols, before the segment sizes: every model of every
segment (order 1: all 256 contexts) starts from them instead of 256 ones and adapts by the reference's rules, so short
segments (many waves per frame) stop paying the model's learning cost.
Version 3 (`nclass` > 1 prior classes; not in the reference): segment s of
the frame's n_segments takes prior row floor(s * nclass / n_segments), row c
built like version 2's over the symbols of class c's segments; after
n_segments come uint32 nclass and per class a sparse row -- uint16 m, the m
symbols whose frequency is not 1 (uint8 each), their m frequencies (uint16) --
and the segment sizes as unsigned LEB128 varints (a 4096-symbol segment of DCT
indices is ~20 bytes: a uint32 index would cost +4.8 % of the stream).
With the DCT's subband layout and nclass = 8 a row is about one subband row,
whose statistics differ the most: 4096-symbol segments (1519 waves for a 1080p
frame) then cost about the serial stream's rate.
decompress() of a malformed header returns zeros((10, 10)) like
CBAAC.py:101-102.
"""
from __future__ import annotations

import io
import struct
import threading

import numpy as np

from . import _lib as L
from .device import DeviceBuffer, Stream

FILE_EXTENSION = ".tadpt_arith"
MAGIC = b"VCFT"
VERSION = 1
VERSION_PRIOR = 2
VERSION_CLASSES = 3
DEFAULT_SEG = 1 << 17     # 48 segments for a 1080p frame, 190 for 4K
PRIOR_SEG = 1 << 15       # version 2: 190 segments for 1080p at +2.3 % rate (profiles/r02_tcbaac_prior.jsonl)
CLASS_SEG = 1 << 12       # version 3 (-c TCBAACP): 1519 segments for 1080p
PRIOR_CLASSES = 8         # version 3's prior rows per frame (the 8 subband rows of the 8x8 DCT)


def n_segments(n: int, seg_len: int = DEFAULT_SEG) -> int:
    return int(L.lib().vcf_cbaac_tiled_segments(int(n), int(seg_len)))


class _Scratch:
    """Device buffers reused across calls (grown on demand)."""

    def __init__(self):
        self.bufs = {}

    def get(self, name: str, nbytes: int) -> DeviceBuffer:
        b = self.bufs.get(name)
        if b is None or b.nbytes < nbytes:
            b = DeviceBuffer(max(nbytes, 1))
            self.bufs[name] = b
        return b


class TiledCoder:
    """The GPU calls, with reusable scratch and a stream.

    One coder owns one set of scratch buffers and one stream, so its calls
    are serialised by `lock` (the DCT CoDec's encode_fns/decode_fns call the
    entropy codec from a thread pool): a call's upload, kernels and download
    never interleave with another thread's on the same buffers."""

    def __init__(self, order: int = 0, seg_len: int = DEFAULT_SEG, stream: Stream | None = None,
                 prior: bool = False, nclass: int = 1):
        self.order, self.seg_len, self.prior = int(order), int(seg_len), bool(prior)
        self.nclass = int(nclass)
        if self.prior and self.order > 1:
            raise NotImplementedError("prior-seeded tiled CBAAC: orders 0 and 1")
        if self.nclass < 1 or (self.nclass > 1 and not self.prior):
            raise ValueError("prior classes need prior=True")
        self.stream = stream if stream is not None else Stream()
        self.scratch = _Scratch()
        self.last_prior = None     # the prior table of the last encode (prior=True)
        self.lock = threading.RLock()

    def encode_device(self, sym: DeviceBuffer, n: int, offset: int = 0):
        """Symbols already in HBM -> (segment byte counts, payload bytes);
        with prior=True the frame's prior table is left in self.last_prior
        (read it under self.lock when other threads share the coder)."""
        with self.lock:
            return self._encode_device(sym, n, offset)

    def _encode_device(self, sym: DeviceBuffer, n: int, offset: int = 0):
        lib = L.lib()
        ns = n_segments(n, self.seg_len)
        ws = self.scratch.get("ws", int(lib.vcf_cbaac_tiled_workspace(n, self.seg_len)))
        cap = int(lib.vcf_cbaac_tiled_bound(n, self.seg_len))
        out = self.scratch.get("out", cap)
        sb = self.scratch.get("sizes", 8 * (ns + 1))
        if self.prior and self.nclass > 1:
            K = self.nclass
            pr, hist = self.scratch.get("prior", 512 * K), self.scratch.get("hist", 1024 * K)
            L.call("vcf_cbaac_tiled_prior_classes", sym.address(offset), 1, int(n), int(n), self.seg_len, K, pr.ptr,
                   hist.ptr, self.stream.handle)
            L.call("vcf_cbaac_tiled_encode_classes", sym.address(offset), 1, int(n), int(n), self.order, pr.ptr, K,
                   self.seg_len, out.ptr, cap, sb.ptr, ws.ptr, self.stream.handle)
            self.last_prior = np.empty((K, 256), np.uint16)
            pr.download(self.last_prior, self.stream)
        elif self.prior:
            pr, hist = self.scratch.get("prior", 512), self.scratch.get("hist", 1024)
            L.call("vcf_cbaac_tiled_prior", sym.address(offset), int(n), pr.ptr, hist.ptr, self.stream.handle)
            L.call("vcf_cbaac_tiled_encode_prior", sym.address(offset), int(n), self.order, pr.ptr, self.seg_len,
                   out.ptr, cap, sb.ptr, ws.ptr, self.stream.handle)
            self.last_prior = np.empty(256, np.uint16)
            pr.download(self.last_prior, self.stream)
        else:
            L.call("vcf_cbaac_tiled_encode", sym.address(offset), int(n), self.order, self.seg_len, out.ptr, cap,
                   sb.ptr, ws.ptr, self.stream.handle)
        sizes = np.empty(ns + 1, np.int64)
        sb.download(sizes, self.stream)
        self.stream.synchronize()
        total = int(sizes[-1])
        payload = np.empty(total, np.uint8)
        if total:
            out.download(payload, self.stream)
            self.stream.synchronize()
        return sizes[:-1].copy(), payload.tobytes()

    def encode(self, sym: np.ndarray):
        sym = np.ascontiguousarray(sym, np.uint8).ravel()
        with self.lock:
            buf = self.scratch.get("sym", sym.size)
            if sym.size:
                buf.upload(sym, self.stream)
            return self._encode_device(buf, sym.size)

    def trace(self, sym: np.ndarray) -> np.ndarray:
        """(n, 3) int32: the (low, high, total) handed to the coder per symbol."""
        with self.lock:
            return self._trace(sym)

    def _trace(self, sym: np.ndarray) -> np.ndarray:
        lib = L.lib()
        sym = np.ascontiguousarray(sym, np.uint8).ravel()
        n = sym.size
        ns = n_segments(n, self.seg_len)
        buf = self.scratch.get("sym", n)
        if n:
            buf.upload(sym, self.stream)
        ws = self.scratch.get("ws", int(lib.vcf_cbaac_tiled_workspace(n, self.seg_len)))
        sb = self.scratch.get("sizes", 8 * (ns + 1))
        tr = DeviceBuffer(max(12 * n, 1))
        L.call("vcf_cbaac_tiled_trace", buf.ptr, n, self.order, self.seg_len, tr.ptr, sb.ptr, ws.ptr,
               self.stream.handle)
        out = np.empty((n, 3), np.int32)
        if n:
            tr.download(out, self.stream)
        self.stream.synchronize()
        return out

    def decode_to_device(self, payload: bytes, seg_bytes, n: int, out: DeviceBuffer, prior=None):
        """Enqueue the decode of n symbols into `out` on self.stream (the
        caller synchronises; hold self.lock across this and that wait when
        other threads share the coder)."""
        with self.lock:
            self._decode_to_device(payload, seg_bytes, n, out, prior)

    def _decode_to_device(self, payload: bytes, seg_bytes, n: int, out: DeviceBuffer, prior=None):
        seg_bytes = np.asarray(seg_bytes, np.int64)
        offs = np.zeros(seg_bytes.size + 1, np.int64)
        np.cumsum(seg_bytes, out=offs[1:])
        if int(offs[-1]) != len(payload):
            raise ValueError("segment sizes do not add up to the payload")
        src = self.scratch.get("in", len(payload))
        if len(payload):
            src.upload(np.frombuffer(payload, np.uint8), self.stream)
        ob = self.scratch.get("offs", offs.nbytes)
        ob.upload(offs, self.stream)
        if prior is not None and np.ndim(prior) == 2:   # version 3: prior classes
            prior = check_prior(prior)
            pr = self.scratch.get("prior_in", prior.nbytes)
            pr.upload(prior, self.stream)
            L.call("vcf_cbaac_tiled_decode_classes", src.ptr, ob.ptr, 1, int(n), self.order, pr.ptr, prior.shape[0],
                   self.seg_len, out.ptr, int(n), self.stream.handle)
        elif prior is not None:
            prior = check_prior(prior)
            pr = self.scratch.get("prior_in", 512)
            pr.upload(prior, self.stream)
            L.call("vcf_cbaac_tiled_decode_prior", src.ptr, ob.ptr, int(n), self.order, pr.ptr, self.seg_len,
                   out.ptr, self.stream.handle)
        else:
            L.call("vcf_cbaac_tiled_decode", src.ptr, ob.ptr, int(n), self.order, self.seg_len, out.ptr,
                   self.stream.handle)

    def decode(self, payload: bytes, seg_bytes, n: int, prior=None) -> np.ndarray:
        with self.lock:
            out = self.scratch.get("dec", n)
            self.decode_to_device(payload, seg_bytes, n, out, prior)
            res = np.empty(n, np.uint8)
            if n:
                out.download(res, self.stream)
            self.stream.synchronize()
            return res


def check_prior(prior) -> np.ndarray:
    """256 uint16 frequencies (or nclass rows of them), each >= 1, every row's
    total below the model's max_freq (so the packed 16-bit cumulative counts
    of the GPU model cannot overflow)."""
    prior = np.ascontiguousarray(prior, np.uint16)
    rows = prior.reshape(-1, 256) if prior.ndim in (1, 2) and prior.shape[-1] == 256 else None
    if (rows is None or not 1 <= rows.shape[0] <= 256 or int(prior.min()) < 1
            or int(rows.sum(axis=1, dtype=np.int64).max()) >= 16384):
        raise ValueError("bad prior table")
    return prior


class FrameBatch:
    """Reusable device state for coding `n_frames` frames of `frame_symbols`
    symbols each (the III driver's per-rank chunk), every frame's code-stream
    kept in HBM.  One launch per stage codes all the frames
    (vcf_cbaac_tiled_*_frames): a frame's few hundred segments alone leave most
    of the chip idle, a batch's segments fill it (and from ~5000 on, order 0
    codes one segment per lane).  Frame f's packed segments sit at byte
    f * cap of `out`, its segment sizes and prior in one contiguous device
    array each, so one download returns the index.  launch() enqueues,
    sizes() waits and downloads the index, payload(f) / download() hand out
    the code-streams."""

    def __init__(self, n_frames: int, frame_symbols: int, order: int = 0, seg_len: int = PRIOR_SEG,
                 prior: bool = True, streams: int | None = None, nclass: int = 1):
        lib = L.lib()
        self.n_frames, self.n = int(n_frames), int(frame_symbols)
        self.order, self.seg_len, self.prior = int(order), int(seg_len), bool(prior)
        self.nclass = int(nclass)
        if self.prior and self.order > 1:
            raise NotImplementedError("prior-seeded tiled CBAAC: orders 0 and 1")
        if self.nclass < 1 or (self.nclass > 1 and not self.prior):
            raise ValueError("prior classes need prior=True")
        self.ns = n_segments(self.n, self.seg_len)
        self.cap = int(lib.vcf_cbaac_tiled_bound(self.n, self.seg_len))
        self.stream = Stream()
        nf = max(self.n_frames, 1)
        self.ws = DeviceBuffer(max(int(lib.vcf_cbaac_tiled_frames_workspace(nf, self.n, self.seg_len)), 1))
        self.out = DeviceBuffer(max(self.cap * nf, 1))
        self.sizes_dev = DeviceBuffer(8 * (self.ns + 1) * nf)
        self.prior_dev = DeviceBuffer(512 * nf * self.nclass)
        self.hist = DeviceBuffer(1024 * nf * self.nclass)
        self._sizes = None
        self._priors = None

    def launch(self, sym: DeviceBuffer, offset: int = 0, after: Stream | None = None,
               frame_stride: int | None = None) -> None:
        """Enqueue frame f = symbols [offset + f * frame_stride, + n) of `sym`
        (frame_stride defaults to n); `after` (the producer's stream) is
        waited for through an event."""
        from .device import Event
        if after is not None:
            ev = Event()
            ev.record(after)
            self.stream.wait_event(ev)
        self._sizes = None
        if not self.n_frames:
            return
        stride = self.n if frame_stride is None else int(frame_stride)
        base = sym.address(offset)
        h = self.stream.handle
        if self.nclass > 1:
            L.call("vcf_cbaac_tiled_prior_classes", base, self.n_frames, self.n, stride, self.seg_len, self.nclass,
                   self.prior_dev.ptr, self.hist.ptr, h)
            L.call("vcf_cbaac_tiled_encode_classes", base, self.n_frames, self.n, stride, self.order,
                   self.prior_dev.ptr, self.nclass, self.seg_len, self.out.ptr, self.cap, self.sizes_dev.ptr,
                   self.ws.ptr, h)
            return
        if self.prior:
            L.call("vcf_cbaac_tiled_prior_frames", base, self.n_frames, self.n, stride, self.prior_dev.ptr,
                   self.hist.ptr, h)
        L.call("vcf_cbaac_tiled_encode_frames", base, self.n_frames, self.n, stride, self.order,
               self.prior_dev.ptr if self.prior else None, self.seg_len, self.out.ptr, self.cap, self.sizes_dev.ptr,
               self.ws.ptr, h)

    def join(self, stream: Stream) -> None:
        """`stream` waits for the coding (no host synchronisation)."""
        from .device import Event
        ev = Event()
        ev.record(self.stream)
        stream.wait_event(ev)

    def sizes(self):
        """Wait for the coding; -> (per-frame segment byte counts (n_frames x
        ns int64), per-frame payload bytes, priors (n_frames x 256) or None)."""
        if self._sizes is None:
            allz = np.empty((self.n_frames, self.ns + 1), np.int64)
            self._priors = None
            if self.n_frames:
                self.sizes_dev.download(allz, self.stream)
                if self.prior:
                    shp = (self.n_frames, self.nclass, 256) if self.nclass > 1 else (self.n_frames, 256)
                    self._priors = np.empty(shp, np.uint16)
                    self.prior_dev.download(self._priors, self.stream)
            self.stream.synchronize()
            self._sizes = allz
        return self._sizes[:, :-1], self._sizes[:, -1].copy(), self._priors

    def payload(self, f: int):
        """(device buffer, byte offset, byte count) of frame f's packed segments."""
        _, totals, _ = self.sizes()
        return self.out, f * self.cap, int(totals[f])

    def header(self, f: int, shape) -> bytes:
        """Frame f's container bytes in front of its payload (pack() minus the payload)."""
        seg, _, pri = self.sizes()
        return pack(tuple(shape), self.order, self.seg_len, seg[f], b"", None if pri is None else pri[f])

    def headers(self, shape) -> list:
        """Every frame's header (== header(f, shape)), built for the whole
        batch at once: version 3's varint indexes and sparse prior rows as a
        few array operations over all frames instead of a pack() per frame."""
        seg, _, pri = self.sizes()
        if pri is None or pri.ndim != 3:
            return [self.header(f, shape) for f in range(self.n_frames)]
        F, K = pri.shape[:2]
        fixed = (np.array([len(shape), *shape], np.uint32).tobytes() + MAGIC +
                 struct.pack("<IIII", VERSION_CLASSES, self.order, self.seg_len, self.ns))
        if int(pri.min()) < 1 or int(pri.sum(axis=2, dtype=np.int64).max()) >= 16384:   # check_prior, every frame
            raise ValueError("bad prior table")
        rb, rend = _sparse_rows_batch(pri)
        vb, vend = _varints_rows(seg)
        rst = np.concatenate([[0], rend[:-1]])
        vst = np.concatenate([[0], vend[:-1]])
        return [fixed + rb[rst[f]:rend[f]] + vb[vst[f]:vend[f]] for f in range(F)]

    def download(self):
        """-> [(segment byte counts, payload bytes, prior or None)] per frame."""
        seg, totals, pri = self.sizes()
        res = []
        for f in range(self.n_frames):
            payload = np.empty(int(totals[f]), np.uint8)
            if payload.size:
                self.out.download(payload, offset=f * self.cap)
            res.append((seg[f].copy(), payload.tobytes(), None if pri is None else pri[f].copy()))
        return res


def encode_frames_device(sym: DeviceBuffer, n_frames: int, frame_symbols: int, order: int = 0,
                         seg_len: int = DEFAULT_SEG, prior: bool = False, streams: int = 4,
                         after: Stream | None = None, offset: int = 0, nclass: int = 1):
    """Several frames' symbols, back to back in HBM from `offset`, each coded
    as its own tiled stream (its own prior with prior=True), all of them in
    one launch per stage (FrameBatch; `streams` is accepted for the earlier
    interface and unused).  `after`: the stream that produced the symbols
    (e.g. the DCT encode's); the coder waits for its work so far (an event),
    so the caller need not synchronise it first.
    -> [(segment byte counts, payload, prior or None)]."""
    fb = FrameBatch(n_frames, frame_symbols, order, seg_len, prior, nclass=nclass)
    fb.launch(sym, offset, after)
    return fb.download()


def _varints_rows(v: np.ndarray):
    """Unsigned LEB128 varints (7 bits per byte, high bit = more) of each row
    of a 2-D array (vcf_leb128_encode_rows) -> (bytes, end offset of each row)."""
    v = np.ascontiguousarray(v, np.int64)
    out = np.empty(max(5 * v.size, 1), np.uint8)
    ends = np.zeros(v.shape[0], np.int64)
    L.call("vcf_leb128_encode_rows", v.ctypes.data, v.shape[0], v.shape[1], out.ctypes.data, out.size,
           ends.ctypes.data)
    return out[:int(ends[-1]) if ends.size else 0].tobytes(), ends


def _varints(v: np.ndarray) -> bytes:
    return _varints_rows(np.asarray(v, np.int64).reshape(1, -1))[0]


def _sparse_rows_batch(pri: np.ndarray):
    """Version 3's sparse prior rows of every frame of an (F, K, 256) array
    (vcf_prior_rows_sparse) -> (bytes, end offset of each frame)."""
    pri = np.ascontiguousarray(pri, np.uint16)
    F, K = pri.shape[:2]
    out = np.empty(F * (4 + K * (2 + 3 * 256)), np.uint8)
    ends = np.zeros(F, np.int64)
    L.call("vcf_prior_rows_sparse", pri.ctypes.data, F, K, out.ctypes.data, out.size, ends.ctypes.data)
    return out[:int(ends[-1]) if F else 0].tobytes(), ends


def _parse_varints(data: bytes, p: int, count: int):
    """-> (count values, the offset after them); ValueError if the data end first."""
    if count == 0:
        return np.zeros(0, np.int64), p
    raw = np.frombuffer(data, np.uint8, min(len(data) - p, 5 * count), p)
    ends = np.flatnonzero(raw < 0x80)
    if ends.size < count:
        raise ValueError("segment index")
    stop = int(ends[count - 1]) + 1
    raw = raw[:stop].astype(np.uint64)
    grp = np.concatenate([[0], np.cumsum(raw[:-1] < 0x80)])
    start = np.concatenate([[0], ends[:count - 1] + 1])
    pos = np.arange(stop) - start[grp]
    if int(pos.max()) > 4:
        raise ValueError("segment index")
    vals = np.zeros(count, np.uint64)
    np.add.at(vals, grp, (raw & np.uint64(0x7F)) << (np.uint64(7) * pos.astype(np.uint64)))
    return vals.astype(np.int64), p + stop


def _sparse_rows(prior: np.ndarray) -> bytes:
    """Version 3's prior rows: per row uint16 m, m uint8 symbols, m uint16 frequencies (those != 1)."""
    return _sparse_rows_batch(np.asarray(prior)[None])[0]


def _parse_sparse_rows(data: bytes, p: int):
    (K,) = struct.unpack_from("<I", data, p)
    if not 1 <= K <= 256:
        raise ValueError(f"{K} prior classes")
    p += 4
    prior = np.ones((K, 256), np.uint16)
    for c in range(K):
        (m,) = struct.unpack_from("<H", data, p)
        if m > 256 or p + 2 + 3 * m > len(data):
            raise ValueError("prior row")
        sy = np.frombuffer(data, np.uint8, m, p + 2)
        prior[c, sy] = np.frombuffer(data, "<u2", m, p + 2 + m)
        p += 2 + 3 * m
    return check_prior(prior), p


def pack(shape, order: int, seg_len: int, seg_bytes, payload: bytes, prior=None) -> bytes:
    """The container: version 1 (prior None), 2 (one 256-entry prior) or 3 (nclass x 256 priors)."""
    seg_bytes = np.asarray(seg_bytes, np.int64)
    head = np.array([len(shape), *shape], np.uint32).tobytes()
    classes = prior is not None and np.ndim(prior) == 2
    version = VERSION if prior is None else (VERSION_CLASSES if classes else VERSION_PRIOR)
    head += MAGIC + struct.pack("<IIII", version, order, seg_len, seg_bytes.size)
    if classes:   # version 3: sparse prior rows, the segment sizes as LEB128 varints
        return head + _sparse_rows(check_prior(prior)) + _varints(seg_bytes) + payload
    if prior is not None:
        head += check_prior(prior).astype("<u2").tobytes()
    head += seg_bytes.astype(np.uint32).tobytes()
    return head + payload


def unpack(data: bytes):
    """-> (shape, order, seg_len, seg_bytes, payload); ValueError if malformed."""
    return _parse(data)[:5]


def _parse(data: bytes):
    """-> (shape, order, seg_len, seg_bytes, payload, prior or None)."""
    nd = struct.unpack_from("<I", data, 0)[0]
    if nd > 16:
        raise ValueError("ndims")
    shape = struct.unpack_from(f"<{nd}I", data, 4)
    p = 4 + 4 * nd
    if data[p:p + 4] != MAGIC:
        raise ValueError("not a tiled CBAAC stream")
    version, order, seg_len, ns = struct.unpack_from("<IIII", data, p + 4)
    if version not in (VERSION, VERSION_PRIOR, VERSION_CLASSES):
        raise ValueError(f"version {version}")
    if order > 1:                       # the GPU coder's orders (both versions)
        raise ValueError(f"order {order}")
    if seg_len <= 0 or seg_len % 256:   # vcf_cbaac_tiled_*: a positive multiple of 256
        raise ValueError(f"segment length {seg_len}")
    p += 20
    prior = None
    if version == VERSION_PRIOR:
        prior = check_prior(np.frombuffer(data, "<u2", 256, p))
        p += 512
    if version == VERSION_CLASSES:
        prior, p = _parse_sparse_rows(data, p)
        seg_bytes, p = _parse_varints(data, p, ns)
    else:
        seg_bytes = np.frombuffer(data, np.uint32, ns, p).astype(np.int64)
        p += 4 * ns
    payload = data[p:]
    n = int(np.prod(shape)) if nd else 1
    if n_segments(n, seg_len) != ns or int(seg_bytes.sum()) != len(payload):
        raise ValueError("segment index does not match the payload")
    return tuple(int(s) for s in shape), int(order), int(seg_len), seg_bytes, payload, prior


class TiledCBAACCodec:
    """The entropy-codec surface of CBAAC.CoDec (compress/decompress,
    file_extension; CBAAC.py:72-156) over the tiled GPU coder."""

    file_extension = FILE_EXTENSION

    def __init__(self, order: int = 0, seg_len: int = DEFAULT_SEG, prior: bool = False, nclass: int = 1):
        self.ORDER = int(order)
        self.seg_len = int(seg_len)
        self.prior = bool(prior)
        self.nclass = int(nclass)
        self._coder = None
        self._make = threading.Lock()

    @property
    def coder(self) -> TiledCoder:
        with self._make:
            if self._coder is None:
                self._coder = TiledCoder(self.ORDER, self.seg_len, prior=self.prior, nclass=self.nclass)
            return self._coder

    def compress(self, img: np.ndarray, fn=None) -> io.BytesIO:
        img = np.asarray(img)
        flat = img.ravel()
        if flat.size and (flat.min() < 0 or flat.max() > 255):
            raise ValueError("CBAAC codes byte symbols (0..255)")
        coder = self.coder
        with coder.lock:    # last_prior belongs to this call's encode
            sizes, payload = coder.encode(flat.astype(np.uint8))
            prior = coder.last_prior if self.prior else None
        b = io.BytesIO(pack(img.shape, self.ORDER, self.seg_len, sizes, payload, prior))
        b.seek(0)
        return b

    def compress_device(self, k: DeviceBuffer, shape, offset: int = 0) -> io.BytesIO:
        """Indices already in HBM (e.g. the DCT encode's output): only the
        compressed bytes cross PCIe."""
        n = int(np.prod(shape))
        coder = self.coder
        with coder.lock:
            sizes, payload = coder.encode_device(k, n, offset)
            prior = coder.last_prior if self.prior else None
        b = io.BytesIO(pack(tuple(shape), self.ORDER, self.seg_len, sizes, payload, prior))
        b.seek(0)
        return b

    def decompress(self, data, fn=None) -> np.ndarray:
        if isinstance(data, io.BytesIO):
            data = data.getvalue()
        data = bytes(data)
        try:
            shape, order, seg_len, seg_bytes, payload, prior = _parse(data)
        except (ValueError, struct.error):
            return np.zeros((10, 10), np.uint8)      # CBAAC.py:101-102
        coder = self.coder if (order, seg_len) == (self.ORDER, self.seg_len) else TiledCoder(order, seg_len)
        n = int(np.prod(shape))
        return coder.decode(payload, seg_bytes, n, prior).reshape(shape)


def host_segments(sym: np.ndarray, order: int = 0, seg_len: int = DEFAULT_SEG):
    """The host serial coder (vcf_cbaac_encode) run on every segment: what
    each segment of the tiled stream must equal (tests, rate reports)."""
    from .cbaac import encode_symbols
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    return [encode_symbols(sym[i:i + seg_len], order) for i in range(0, sym.size, seg_len)]


def prior_of(sym: np.ndarray, nclass: int = 1, seg_len: int | None = None) -> np.ndarray:
    """The version-2 prior of a frame's symbols (nclass = 1), or version 3's
    nclass rows for segments of seg_len, on the host (what
    vcf_cbaac_tiled_prior / _prior_classes compute on the GPU)."""
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    if nclass == 1:
        hist = np.bincount(sym, minlength=256).astype(np.uint64)
        n = max(sym.size, 1)
        return (1 + hist * 8192 // n).astype(np.uint16)
    ns = n_segments(sym.size, seg_len)
    rows = np.ones((nclass, 256), np.uint16)
    for c in range(nclass):
        segs = [s for s in range(ns) if s * nclass // ns == c]
        if not segs:
            continue
        part = sym[segs[0] * seg_len:(segs[-1] + 1) * seg_len]
        hist = np.bincount(part, minlength=256).astype(np.uint64)
        rows[c] = (1 + hist * 8192 // max(part.size, 1)).astype(np.uint16)
    return rows


def host_segments_prior(sym: np.ndarray, prior, seg_len: int = DEFAULT_SEG, order: int = 0):
    """vcf_cbaac_encode_prior on every segment: what each segment of a
    version-2 stream (one prior) or version-3 stream (prior rows: segment s of
    ns takes row s * nclass // ns) must equal."""
    import ctypes
    prior = check_prior(prior)
    sym = np.ascontiguousarray(sym, np.uint8).ravel()
    lib = L.lib()
    res = []
    ns = n_segments(sym.size, seg_len)
    for i in range(0, sym.size, seg_len):
        seg = np.ascontiguousarray(sym[i:i + seg_len])
        row = np.ascontiguousarray(prior[(i // seg_len) * prior.shape[0] // ns]) if prior.ndim == 2 else prior
        cap = int(lib.vcf_cbaac_bound(seg.size))
        out = np.empty(cap, np.uint8)
        nb, bits = ctypes.c_int64(), ctypes.c_int64()
        L.call("vcf_cbaac_encode_prior", seg.ctypes.data, seg.size, order, row.ctypes.data, out.ctypes.data, cap,
               ctypes.byref(nb), ctypes.byref(bits))
        res.append(out[:nb.value].tobytes())
    return res


def host_decode_prior(data: bytes, n: int, prior, order: int = 0) -> np.ndarray:
    prior = check_prior(prior)
    out = np.empty(n, np.uint8)
    buf = np.frombuffer(data, np.uint8)
    L.call("vcf_cbaac_decode_prior", buf.ctypes.data if buf.size else None, buf.size, n, order, prior.ctypes.data,
           out.ctypes.data)
    return out
