"""Host-side rendezvous for one-process-per-GPU runs (no PyTorch).

The III / IPP drivers and bench.py run one process per GPU.
They need very little from the host side: a barrier, the max / sum of a few
scalars, and the exchange of a small blob (the RCCL unique id, per-frame
code-stream sizes).  `HostGroup` does exactly that over TCP: rank 0 serves on
MASTER_ADDR:port, every rank sends its blob for collective number `seq`, rank
0 answers each rank with all `world` blobs once they are in.  Payload bytes
of the data path never go through here: they move over RCCL
(`vcf_amd.rccl.Communicator`), this group only bootstraps it.

Environment (torch.distributed.run's names, so either launcher works):
RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR (default 127.0.0.1), MASTER_PORT.
The store listens on VCF_STORE_PORT if set, else MASTER_PORT + 1 (torchrun's
own store already holds MASTER_PORT).
"""
from __future__ import annotations

import os
import socket
import struct
import time

__all__ = ["env_world", "HostGroup", "free_port"]


def env_world():
    """(rank, world, local_rank) from the launcher's environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port(host: str = "127.0.0.1") -> int:
    """An unused TCP port (for launchers that pick MASTER_PORT themselves)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _send(sock: socket.socket, data: bytes) -> None:
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("host store: peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class HostGroup:
    """All-gather of small host blobs among `world` processes (rank 0 serves).

    Every collective is an all-gather; barrier / allreduce / broadcast are
    built on it.  Blobs are plain bytes (scalars travel as little-endian f64).
    """

    def __init__(self, rank: int | None = None, world: int | None = None,
                 addr: str | None = None, port: int | None = None, timeout: float = 300.0):
        r, w, _ = env_world()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.timeout = timeout
        self._seq = 0
        self._server = None
        self._conns = []
        if self.world <= 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            if "VCF_STORE_PORT" in os.environ:
                port = int(os.environ["VCF_STORE_PORT"])
            else:
                port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(timeout)
            self._server = srv
            conns = [None] * self.world
            for _ in range(self.world - 1):
                c, _a = srv.accept()
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(timeout)
                (peer,) = struct.unpack("<i", _recv_exact(c, 4))
                if not 0 < peer < self.world or conns[peer] is not None:
                    raise RuntimeError(f"host store: unexpected rank {peer}")
                conns[peer] = c
            self._conns = conns
        else:
            deadline = time.monotonic() + timeout
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.settimeout(timeout)
            c.sendall(struct.pack("<i", self.rank))
            self._conns = [c]

    # -- the one collective ---------------------------------------------------------
    def all_gather_bytes(self, blob: bytes) -> list:
        """Every rank's blob, in rank order, on every rank."""
        if self.world <= 1:
            return [bytes(blob)]
        self._seq += 1
        if self.rank == 0:
            blobs = [bytes(blob)] + [None] * (self.world - 1)
            for r in range(1, self.world):
                blobs[r] = _recv(self._conns[r])
            packed = b"".join(struct.pack("<Q", len(b)) + b for b in blobs)
            for r in range(1, self.world):
                _send(self._conns[r], packed)
            return blobs
        _send(self._conns[0], bytes(blob))
        packed = _recv(self._conns[0])
        out, off = [], 0
        for _ in range(self.world):
            (n,) = struct.unpack_from("<Q", packed, off)
            off += 8
            out.append(packed[off:off + n])
            off += n
        return out

    # -- helpers ----------------------------------------------------------------------
    def barrier(self) -> None:
        self.all_gather_bytes(b"")

    def all_gather_f64(self, v: float) -> list:
        return [struct.unpack("<d", b)[0] for b in self.all_gather_bytes(struct.pack("<d", float(v)))]

    def allreduce_max(self, v: float) -> float:
        return max(self.all_gather_f64(v))

    def allreduce_sum(self, v: float) -> float:
        return float(sum(self.all_gather_f64(v)))

    def broadcast_bytes(self, blob: bytes | None, root: int = 0) -> bytes:
        return self.all_gather_bytes(blob if self.rank == root else b"")[root]

    def close(self) -> None:
        for c in self._conns:
            if c is not None:
                try:
                    c.close()
                except OSError:
                    pass
        self._conns = []
        if self._server is not None:
            self._server.close()
            self._server = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

