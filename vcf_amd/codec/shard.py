"""Frame sharding for the III / IPP drivers.

Frames of a sequence are independent units (intra-only coding; every model
and state resets per frame in encode_fn/decode_fn), so N frames split into P
contiguous chunks, frame i on rank floor(i * P / N), with no collective on
the data path.  The one exchange step is after coding: an all-gather of the
per-frame code-stream sizes (int64) and, when the code-streams must end up
on rank 0 (no shared filesystem), a gather of the variable-length payloads
to rank 0 -- RCCL has no gatherv, so libvcf_amd.so's `vcf_comm_gatherv`
posts one send per peer and P-1 concurrent receives on the root: on xGMI
each peer has its own link to rank 0, the step is link-bound, not
ring-bound.  This replaces the point where the reference's sequential frame
loop holds every coded frame in one process (src/III.py:77-115, :132-144).

One process per GPU: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT come from the launcher (torch.distributed.run's names; any
launcher that sets them works).  Backends:
- "rccl" (default when the ranks see a GPU): sizes and payloads over RCCL
  through vcf_amd.rccl.Communicator;
- "host": the TCP host group carries them (CPU tests only -- no GPU there).
The host group (vcf_amd/comm.py) bootstraps RCCL and carries the barrier
either way.  No PyTorch.
"""
from __future__ import annotations

import numpy as np

from ..comm import HostGroup, env_world


def frame_range(n_frames: int, rank: int, world: int):
    """Contiguous chunk of frames owned by `rank`: i with floor(i*P/N) == rank."""
    lo = (rank * n_frames + world - 1) // world
    hi = ((rank + 1) * n_frames + world - 1) // world
    return lo, min(hi, n_frames)


def owner(i: int, n_frames: int, world: int) -> int:
    return i * world // n_frames


def _gpu_count() -> int:
    from ..device import device_count
    try:
        return device_count()
    except Exception:      # no ROCm device in this process (CPU tests)
        return 0


class Group:
    """The ranks of a frame-sharded job (or the trivial single-rank one)."""

    def __init__(self, backend: str | None = None):
        self.rank, self.world, self.local = env_world()
        self.host = None
        self.comm = None
        self.backend = None
        if self.world <= 1:
            return
        ndev = _gpu_count() if backend in (None, "rccl") else 0
        if backend is None:
            backend = "rccl" if ndev > 0 else "host"
        if backend not in ("rccl", "host"):
            raise ValueError(f"backend {backend!r}: 'rccl' or 'host'")
        self.host = HostGroup(self.rank, self.world)
        self.backend = backend
        if backend == "rccl":
            if ndev <= 0:
                raise RuntimeError("backend 'rccl' needs a GPU in every rank")
            from ..device import set_device
            from ..rccl import Communicator
            set_device(self.local % ndev)
            self.comm = Communicator(self.host)

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def all_gather_sizes(self, n_frames: int, local_sizes) -> np.ndarray:
        """Per-frame sizes (int64, length n_frames) on every rank."""
        mine = np.asarray(local_sizes, np.int64)
        if not self.distributed:
            return mine.copy()
        lo, hi = frame_range(n_frames, self.rank, self.world)
        if mine.size != hi - lo:
            raise ValueError(f"rank {self.rank} owns frames {lo}..{hi} but reports {mine.size} sizes")
        full = np.zeros(n_frames, np.int64)
        full[lo:hi] = mine
        if self.comm is not None:
            rows = self.comm.all_gather_i64(full)
        else:
            rows = np.stack([np.frombuffer(b, np.int64) for b in self.host.all_gather_bytes(full.tobytes())])
        out = np.zeros(n_frames, np.int64)
        for r in range(self.world):                  # each rank fills only its own chunk
            rlo, rhi = frame_range(n_frames, r, self.world)
            out[rlo:rhi] = rows[r, rlo:rhi]
        return out

    def gather_payloads(self, n_frames: int, local_payloads, sizes: np.ndarray):
        """Rank 0 receives every frame's code-stream bytes (list of bytes,
        frame order); other ranks return None.  `sizes` from all_gather_sizes."""
        if not self.distributed:
            return [bytes(p) for p in local_payloads]
        sizes = np.asarray(sizes, np.int64)
        lo, hi = frame_range(n_frames, self.rank, self.world)
        blob = b"".join(bytes(p) for p in local_payloads)
        if len(blob) != int(sizes[lo:hi].sum()):
            raise ValueError("local payload bytes disagree with the gathered sizes")
        if self.comm is not None:
            counts = np.array([sizes[slice(*frame_range(n_frames, r, self.world))].sum()
                               for r in range(self.world)], np.int64)
            packed = self.comm.gatherv(blob, counts, root=0)
            if self.rank != 0:
                return None
            packed = packed.tobytes()
        else:
            blobs = self.host.all_gather_bytes(blob if self.rank != 0 else b"")
            if self.rank != 0:
                return None
            packed = blob + b"".join(blobs[1:])
        out, off = [], 0
        for i in range(n_frames):
            out.append(packed[off:off + int(sizes[i])])
            off += int(sizes[i])
        return out

    def gather_blobs(self, blob: bytes):
        """Rank 0: every rank's blob in rank order (item r belongs to rank r)."""
        if not self.distributed:
            return [bytes(blob)]
        sizes = self.all_gather_sizes(self.world, [len(blob)])
        return self.gather_payloads(self.world, [blob], sizes)

    def barrier(self):
        if self.host is not None:
            self.host.barrier()

    def close(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None
        if self.host is not None:
            self.host.close()
            self.host = None
