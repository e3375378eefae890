"""RCCL communicator over libvcf_amd.so's vcf_comm_* C ABI (no PyTorch).

One process per GPU.  The unique id is created by rank 0
(`vcf_comm_unique_id`) and handed to the other ranks through the host group
(vcf_amd/comm.py); after that every byte moves over RCCL on xGMI.

Every call is bounded: the communicator is non-blocking (vcf_comm_init_timeout)
and every wait goes through vcf_comm_wait, so a peer that never arrives ends
the call with VCFTimeout (the communicator aborted) instead of a hang.  The
timeout is `timeout_s`, else VCF_COMM_TIMEOUT_MS from the environment, else
120 s.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from ._lib import call
from .comm import HostGroup
from .device import DeviceBuffer, Stream

ID_BYTES = 128


class _stdout_to_stderr:
    """fd 1 -> fd 2 for the duration (output of C code in this process)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False
SUM, MAX, MIN = 0, 1, 2


class Communicator:
    """An RCCL communicator over the ranks of `host` (device already set)."""

    def __init__(self, host: HostGroup, timeout_s: float | None = None):
        self.rank, self.world = host.rank, host.world
        uid = (ctypes.c_uint8 * ID_BYTES)()
        if self.rank == 0:
            call("vcf_comm_unique_id", uid, ID_BYTES)
        blob = host.broadcast_bytes(bytes(uid) if self.rank == 0 else None)
        uid = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(blob)
        h = ctypes.c_void_p()
        self.handle = None
        with _stdout_to_stderr():    # RCCL prints its version banner on stdout; bench.py's stdout is one JSON line
            call("vcf_comm_init_timeout", ctypes.byref(h), uid, self.rank, self.world,
                 int(timeout_s * 1000) if timeout_s else 0)
        self.handle = h
        self.stream = Stream()

    def wait(self, stream: Stream | None = None) -> None:
        """Wait for `stream` (default: the communicator's) within the timeout."""
        call("vcf_comm_wait", self.handle, (stream or self.stream).handle)

    # -- collectives (host arrays in, host arrays out; staged through HBM) ----------------
    def all_gather_i64(self, values) -> np.ndarray:
        """(world, n) int64: row r = rank r's `values` (same length on every rank)."""
        a = np.ascontiguousarray(values, dtype=np.int64).ravel()
        n = a.size
        if n == 0:
            return np.zeros((self.world, 0), np.int64)
        src = DeviceBuffer.from_array(a, self.stream)
        dst = DeviceBuffer(a.nbytes * self.world)
        call("vcf_comm_allgather_i64", self.handle, src.ptr, n, dst.ptr, self.stream.handle)
        out = np.empty((self.world, n), np.int64)
        dst.download(out, self.stream)
        self.wait()
        return out

    def allreduce_f64(self, values, op: int = SUM) -> np.ndarray:
        a = np.ascontiguousarray(values, dtype=np.float64).ravel()
        if a.size == 0:
            return a.copy()
        src = DeviceBuffer.from_array(a, self.stream)
        dst = DeviceBuffer(a.nbytes)
        call("vcf_comm_allreduce_f64", self.handle, src.ptr, dst.ptr, a.size, op, self.stream.handle)
        out = np.empty_like(a)
        dst.download(out, self.stream)
        self.wait()
        return out

    def gatherv(self, data, counts, root: int = 0):
        """Rank r's bytes (counts[r] of them) packed in rank order on `root`
        (a uint8 array there, None elsewhere).  Host bytes in: staged to HBM."""
        counts = self._counts(counts)
        mine = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
            np.ascontiguousarray(data).view(np.uint8).ravel()
        if mine.size != counts[self.rank]:
            raise ValueError(f"rank {self.rank} sends {mine.size} bytes, counts says {counts[self.rank]}")
        total = int(counts.sum())
        src = DeviceBuffer.from_array(mine, self.stream) if mine.size else None
        dst = DeviceBuffer(total) if self.rank == root and total else None
        self.gatherv_device(src, int(mine.size), counts, dst, root)
        out = None
        if self.rank == root:
            out = np.empty(total, np.uint8)
            if total:
                dst.download(out, self.stream)
        self.wait()
        return out

    def gatherv_device(self, src: DeviceBuffer | None, nbytes: int, counts, dst: DeviceBuffer | None,
                       root: int = 0, src_offset: int = 0, stream: Stream | None = None) -> None:
        """Device to device: `nbytes` of `src` (from src_offset) land packed in
        rank order in `dst` on `root` (code-streams already in HBM, e.g. the
        tiled CBAAC's output, never cross PCIe).  Enqueued on `stream`
        (default: the communicator's); the caller waits with wait()."""
        counts = self._counts(counts)
        total = int(counts.sum())
        if self.rank == root and total and (dst is None or dst.nbytes < total):
            raise ValueError("root needs a receive buffer of sum(counts) bytes")
        if nbytes and (src is None or src.nbytes < src_offset + nbytes):
            raise ValueError("send buffer smaller than nbytes")
        call("vcf_comm_gatherv", self.handle, src.address(src_offset) if (src is not None and nbytes) else None,
             int(nbytes), dst.ptr if (dst is not None and self.rank == root) else None,
             counts.ctypes.data_as(ctypes.c_void_p), root, (stream or self.stream).handle)

    def _counts(self, counts) -> np.ndarray:
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        if counts.size != self.world:
            raise ValueError("counts needs one entry per rank")
        return counts

    def close(self) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            call("vcf_comm_destroy", self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
