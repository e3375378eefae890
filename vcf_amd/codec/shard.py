"""Frame sharding for the III driver.

Frames of a sequence are independent units (intra-only coding; every model
and state resets per frame in encode_fn/decode_fn), so N frames split into P
contiguous chunks, frame i on rank floor(i * P / N), with no collective on
the data path.  The one exchange step is after coding: an all-gather of the
per-frame code-stream sizes (int64) and, when the code-streams must end up
on rank 0 (no shared filesystem), point-to-point sends of the variable-length
payloads to rank 0 -- RCCL has no gatherv, and on xGMI each peer has its own
link to rank 0, so P-1 concurrent sends are link-bound, not ring-bound.

One process per GPU: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR come from
torch.distributed.run; backend "nccl" (= RCCL) when the ranks own GPUs,
"gloo" otherwise (the CPU tests).
"""
from __future__ import annotations

import os

import numpy as np


def env_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def frame_range(n_frames: int, rank: int, world: int):
    """Contiguous chunk of frames owned by `rank`: i with floor(i*P/N) == rank."""
    lo = (rank * n_frames + world - 1) // world
    hi = ((rank + 1) * n_frames + world - 1) // world
    return lo, min(hi, n_frames)


def owner(i: int, n_frames: int, world: int) -> int:
    return i * world // n_frames


class Group:
    """A torch.distributed process group (or the trivial single-rank one)."""

    def __init__(self, backend: str | None = None):
        self.rank, self.world, self.local = env_world()
        self.dist = None
        self.device = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if not dist.is_initialized():
                dist.init_process_group(backend, rank=self.rank, world_size=self.world)
            self.dist = dist
            self.backend = backend
            self.device = torch.device("cuda", self.local) if backend == "nccl" else torch.device("cpu")
        else:
            self.backend = None

    def _t(self, a):
        import torch
        return torch.as_tensor(a).to(self.device)

    def all_gather_sizes(self, n_frames: int, local_sizes) -> np.ndarray:
        """Per-frame sizes (int64, length n_frames) on every rank."""
        if self.dist is None:
            return np.asarray(local_sizes, np.int64)
        import torch
        full = np.zeros(n_frames, np.int64)
        lo, hi = frame_range(n_frames, self.rank, self.world)
        full[lo:hi] = np.asarray(local_sizes, np.int64)
        t = self._t(full)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)   # disjoint chunks: sum == gather
        return t.cpu().numpy().astype(np.int64)

    def gather_payloads(self, n_frames: int, local_payloads, sizes: np.ndarray):
        """Rank 0 receives every frame's code-stream bytes (list of bytes,
        frame order); other ranks return None.  `sizes` from all_gather_sizes."""
        if self.dist is None:
            return list(local_payloads)
        import torch
        lo, hi = frame_range(n_frames, self.rank, self.world)
        if self.rank != 0:
            if hi > lo:
                buf = np.frombuffer(b"".join(local_payloads), np.uint8).copy()
                self.dist.send(self._t(buf), dst=0)
            return None
        out = [None] * n_frames
        for i in range(lo, hi):
            out[i] = bytes(local_payloads[i - lo])
        # post every peer's receive at once: each xGMI peer has its own link to
        # rank 0, so the P-1 transfers run concurrently (link-bound, not serial)
        pending = []
        for r in range(1, self.world):
            rlo, rhi = frame_range(n_frames, r, self.world)
            if rhi <= rlo:
                continue
            t = torch.empty(int(sizes[rlo:rhi].sum()), dtype=torch.uint8, device=self.device)
            pending.append((r, rlo, rhi, t, self.dist.irecv(t, src=r)))
        for r, rlo, rhi, t, req in pending:
            req.wait()
            blob = t.cpu().numpy().tobytes()
            off = 0
            for i in range(rlo, rhi):
                out[i] = blob[off:off + int(sizes[i])]
                off += int(sizes[i])
        return out

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()
