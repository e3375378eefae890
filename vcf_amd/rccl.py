"""RCCL communicator over libvcf_amd.so's vcf_comm_* C ABI (no PyTorch).

One process per GPU.  The unique id is created by rank 0
(`vcf_comm_unique_id`) and handed to the other ranks through the host group
(vcf_amd/comm.py); after that every byte moves over RCCL on xGMI.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call
from .comm import HostGroup
from .device import DeviceBuffer, Stream

ID_BYTES = 128
SUM, MAX, MIN = 0, 1, 2


class Communicator:
    """An RCCL communicator over the ranks of `host` (device already set)."""

    def __init__(self, host: HostGroup):
        self.rank, self.world = host.rank, host.world
        uid = (ctypes.c_uint8 * ID_BYTES)()
        if self.rank == 0:
            call("vcf_comm_unique_id", uid, ID_BYTES)
        blob = host.broadcast_bytes(bytes(uid) if self.rank == 0 else None)
        uid = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(blob)
        h = ctypes.c_void_p()
        call("vcf_comm_init", ctypes.byref(h), uid, self.rank, self.world)
        self.handle = h
        self.stream = Stream()

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
        self.stream.synchronize()
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
        self.stream.synchronize()
        return out

    def gatherv(self, data, counts, root: int = 0):
        """Rank r's bytes (counts[r] of them) packed in rank order on `root`
        (a uint8 array there, None elsewhere)."""
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        if counts.size != self.world:
            raise ValueError("counts needs one entry per rank")
        mine = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
            np.ascontiguousarray(data).view(np.uint8).ravel()
        if mine.size != counts[self.rank]:
            raise ValueError(f"rank {self.rank} sends {mine.size} bytes, counts says {counts[self.rank]}")
        total = int(counts.sum())
        src = DeviceBuffer.from_array(mine, self.stream) if mine.size else None
        dst = DeviceBuffer(total) if self.rank == root and total else None
        call("vcf_comm_gatherv", self.handle, src.ptr if src else None, int(mine.size),
             dst.ptr if dst else None, counts.ctypes.data_as(ctypes.c_void_p), root, self.stream.handle)
        out = None
        if self.rank == root:
            out = np.empty(total, np.uint8)
            if total:
                dst.download(out, self.stream)
        self.stream.synchronize()
        return out

    def close(self) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            call("vcf_comm_destroy", self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
